"""L-layer GCN full-graph training and hipGraph-captured inference -- GNN
track, not in the reference.

``DeepGCNTrainer`` covers the depths / dtypes the fused 2-layer trainer
(``gcn.GCNTrainer``) does not: any number of layers (BASELINE config
"ogbn-arxiv 3-layer GCN full-graph bf16").

* ``fused=True`` (default for bf16 on a GPU; also runs on the CPU through the
  reference branches of the same ops): a hand-scheduled epoch on the HIP kernels
  only -- CSR SpMM (gnn_sparse.hip), the fused MFMA dense layers (gnn_linear.hip:
  bias + ReLU + Philox dropout + row scale in the GEMM epilogue, mask-on-load
  backward, split-K weight gradient), the fused aggregate + cross-entropy
  (``spmm_ce``, loss gradient compact over the train rows) and the flat Adam;
  no autograd, no hipBLASLt, no ATen elementwise / dropout / NLL kernels.
  Every hidden layer aggregates first (``AH = Â H``, the narrower gather) and
  stores its output row-scaled, ``Hs = D^-1/2 dropout(relu(AH W + b))``, which is
  both the next layer's gather source and -- through ``Hs > 0`` -- its own
  ReLU / dropout mask in the backward; the last layer transforms first
  (``Zs = Hs W``, 40-48-wide rows for the gather).  The whole epoch is captured
  into one hipGraph (dropout step read from the device Adam counter).
* ``fused=False``: ``layers.GCNConv`` modules under PyTorch autograd with a
  capturable Adam (any storage dtype; the fp16 / fp32 path).

``GCNInference`` is the latency path (BASELINE config "Reddit 2-layer GCN fp16
single-GPU inference"): weights cast once to the inference dtype, features
pre-scaled by D^-1/2 once (the cached normalisation), bias + ReLU in the SpMM
epilogue, and the whole forward captured into one hipGraph.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

import math

from ..utils.hipgraph import StepGraph
from ..utils.philox import model_key
from . import ops
from .data import GraphData
from .layers import GCN, NormGraph, aggregate, pad_cols
from .linear import lin_bwd_data, lin_bwd_weight, lin_fwd


def _ru(x, m):
    return (x + m - 1) // m * m


def cross_entropy(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy in fp32 as log-sum-exp minus the target logit
    (two row reductions; PyTorch's nll_loss reduces with a single workgroup)."""
    o = logits.float()
    return (torch.logsumexp(o, 1) - o.gather(1, y[:, None]).squeeze(1)).mean()


def _splits(g: GraphData):
    return {k: torch.nonzero(g.mask == v).flatten() for k, v in (("train", 1), ("val", 2), ("test", 3))}


class DeepGCNTrainer:
    def __init__(self, g: GraphData, hidden: int = 256, layers: int = 3, dropout: float = 0.5,
                 lr: float = 0.01, dtype: torch.dtype = torch.bfloat16, seed: int = 0,
                 capture: Optional[bool] = None, fused: Optional[bool] = None, train_rows_only: bool = True):
        self.dev = g.rowptr.device
        cuda = self.dev.type == "cuda"
        if fused is None:
            fused = cuda and dtype == torch.bfloat16
        self.fused = bool(fused) and layers >= 2
        if self.dev.type == "cpu" and dtype != torch.float32 and not self.fused:
            dtype = torch.float32                     # CPU reference path: fp32
        self.dtype = torch.bfloat16 if self.fused else dtype
        self.C = g.n_classes
        self.layers = layers
        self.epoch = 0
        if self.fused:
            self._fused = _FusedDeepGCN(g, hidden, layers, dropout, lr, seed, train_rows_only)
            self._step_graph = StepGraph(self._fused.train_body, enabled=cuda if capture is None else capture and cuda,
                                         device=self.dev)
            return
        self.ng = NormGraph.from_data(g)
        self.x = pad_cols(g.x.float()).to(dtype).contiguous()
        dims = [self.x.shape[1]] + [hidden] * (layers - 1) + [self.C]
        self.model = GCN(dims, dropout, seed).to(self.dev)
        with torch.no_grad():                         # padded feature rows of W1 stay 0
            self.model.convs[0].weight[g.n_features:] = 0
        self.opt = torch.optim.Adam(self.model.parameters(), lr=lr, capturable=cuda)
        self.idx = _splits(g)
        self.y = g.y.long()
        self.y_train = self.y[self.idx["train"]]
        self._step_graph = StepGraph(self._step, enabled=cuda if capture is None else capture and cuda,
                                     device=self.dev)

    def _step(self):
        self.model.train()
        out = self.model(self.x, self.ng)
        loss = cross_entropy(out[self.idx["train"]], self.y_train)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        self.opt.step()
        return loss.detach()

    def train_step(self) -> torch.Tensor:
        """One full-graph epoch; returns the loss as a device scalar (no host sync)."""
        loss = self._step_graph()
        self.epoch += 1
        return loss

    @torch.no_grad()
    def evaluate(self):
        if self.fused:
            return self._fused.evaluate()
        self.model.eval()
        out = self.model(self.x, self.ng).float()
        pred = out.argmax(1)
        res = {"train_loss": float(torch.nn.functional.cross_entropy(out[self.idx["train"]], self.y_train))}
        for k in ("train", "val", "test"):
            i = self.idx[k]
            res[k + "_acc"] = float((pred[i] == self.y[i]).float().mean()) if i.numel() else float("nan")
        return res

    # ---------------------------------------------------------------- checkpoint
    def state_tensors(self):
        if self.fused:
            return self._fused.state_tensors()
        from .checkpoint import module_optimizer_tensors
        return module_optimizer_tensors(self.model, self.opt)

    def load_state_tensors(self, t):
        if self.fused:
            self._fused.load_state_tensors(t)
        else:
            from .checkpoint import load_module_optimizer_tensors
            load_module_optimizer_tensors(self.model, self.opt, t)
        self._step_graph.reset()       # the optimizer state tensors were replaced


class _FusedDeepGCN:
    """The fused L-layer GCN epoch (see the module docstring).  Parameters: one flat
    fp32 buffer [W_1, b_1, ..., W_L, b_L] initialised exactly like ``layers.GCN``
    (glorot-uniform W from the same generator sequence, zero b), Adam moments and a
    device step counter beside it."""

    def __init__(self, g: GraphData, hidden: int, layers: int, dropout: float, lr: float, seed: int,
                 train_rows_only: bool = True):
        dev = g.rowptr.device
        self.dev, self.n, self.L = dev, g.n, layers
        self.F, self.C, self.p, self.lr = g.n_features, g.n_classes, float(dropout), float(lr)
        self.dims = [self.F] + [hidden] * (layers - 1) + [self.C]
        self.rowptr, self.col, self.dinv = g.rowptr.contiguous(), g.col.contiguous(), g.dinv.contiguous()
        self.y = g.y.to(torch.int32).contiguous()
        self.mask = g.mask.contiguous()
        self.n_train = int((g.mask == 1).sum())
        self.n_val = int((g.mask == 2).sum())
        self.n_test = int((g.mask == 3).sum())
        bf = dict(dtype=torch.bfloat16, device=dev)
        n = g.n
        # gathered matrices padded to whole 128-byte rows
        ld = [_ru(d, 64) for d in self.dims]
        self.ld = ld
        self.Xs = torch.zeros(n, ld[0], **bf)
        self.Xs[:, :self.F] = (g.x.float() * g.dinv[:, None]).to(torch.bfloat16)
        # parameters (same init sequence as layers.GCN)
        gen = torch.Generator().manual_seed(seed)
        sizes, self.offs = [], []
        off = 0
        flat_parts = []
        for a, b in zip(self.dims[:-1], self.dims[1:]):
            bound = math.sqrt(6.0 / (a + b))
            W = (torch.rand(a, b, generator=gen) * 2 - 1) * bound
            flat_parts += [W.reshape(-1), torch.zeros(b)]
            self.offs.append((off, off + a * b, off + a * b + b))
            off += a * b + b
        self.params = torch.cat(flat_parts).to(dev)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.W, self.b, self.gW, self.gb = [], [], [], []
        for (o0, o1, o2), a, b in zip(self.offs, self.dims[:-1], self.dims[1:]):
            self.W.append(self.params[o0:o1].view(a, b))
            self.b.append(self.params[o1:o2])
            self.gW.append(self.grads[o0:o1].view(a, b))
            self.gb.append(self.grads[o1:o2])
        self.keys = [model_key(seed, "gcn-dropout", l) for l in range(layers - 1)]
        # activations: AH[l] = Â H_{l-1} (input of hidden layer l), Hs[l] = D^-1/2 H_l
        self.AH = [torch.zeros(n, ld[l], **bf) for l in range(layers - 1)]
        self.Hs = [torch.zeros(n, ld[l + 1], **bf) for l in range(layers - 1)]
        self.Zs = torch.zeros(n, ld[-1], **bf)
        self.dZs = torch.zeros(n, ld[-1], **bf)
        self.dH = torch.zeros(n, ld[-2], **bf)
        self.dAHs = torch.zeros(n, max(ld[1:-1] or [8]), **bf)
        self.gb_scratch = torch.zeros(self.C, dtype=torch.float32, device=dev)
        # compact loss gradient (train rows only) and the adjacency restricted to train columns
        train = (g.mask == 1)
        ordinal = torch.cumsum(train.to(torch.int64), 0) - 1
        self.gslot = torch.where(train, ordinal, torch.full_like(ordinal, -1)).to(torch.int32).contiguous()
        col = self.col.long()
        keep = train[col]
        deg = (self.rowptr[1:] - self.rowptr[:-1]).long()
        rows = torch.repeat_interleave(torch.arange(n, device=dev), deg)
        cnt = torch.bincount(rows[keep], minlength=n)
        rp = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        rp[1:] = torch.cumsum(cnt, 0)
        self.rp_T = rp.to(torch.int32).contiguous()
        self.col_T = self.gslot[col[keep]].contiguous()
        self.Gc = torch.zeros(max(self.n_train, 1), ld[-1], **bf)
        # training epochs: the last aggregation (+ cross-entropy) only at the train rows,
        # the only logits the loss reads (exact; see gcn.GCNTrainer; train_rows_only=False:
        # every row)
        self._tr = None
        trows = torch.nonzero(train).flatten()
        if trows.numel() and train_rows_only:
            rpl = self.rowptr.long()
            lo, dg = rpl[trows], rpl[trows + 1] - rpl[trows]
            # long rows first (a whole wave each in spmm_ce); slot = ascending position
            order, self._tr_long = ops.long_row_order(dg)
            trows, lo, dg = trows[order], lo[order], dg[order]
            trp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
            trp[1:] = torch.cumsum(dg, 0)
            eid = torch.arange(int(trp[-1]), device=dev) + torch.repeat_interleave(lo - trp[:-1], dg)
            self._tr = (trp.to(torch.int32).contiguous(), self.col[eid].contiguous(),
                        self.dinv[trows].contiguous(), self.y[trows].contiguous(), self.mask[trows].contiguous(),
                        order.to(torch.int32).contiguous())
        self.last_stats = None

    def _dropout_step(self):
        return self.step_t if self.dev.type == "cuda" else int(self.step_t.item())

    def forward(self, train: bool):
        L, p = self.L, (self.p if train else 0.0)
        src = self.Xs
        step = self._dropout_step()
        for l in range(L - 1):
            ops.spmm(self.rowptr, self.col, src, self.dims[l], rscale=self.dinv, out=self.AH[l])
            lin_fwd(self.AH[l], self.W[l], self.b[l], K1=self.dims[l], relu=True, p=p, key=self.keys[l], step=step,
                    rscale=self.dinv, out=self.Hs[l])
            src = self.Hs[l]
        lin_fwd(src, self.W[L - 1], None, K1=self.dims[L - 1], out=self.Zs)
        if train and self._tr is not None:
            rp, col, dinv, y, mask, gslot = self._tr
            stats, _ = ops.spmm_ce(rp, col, self.Zs, self.C, dinv, self.b[L - 1], y, mask,
                                   1.0 / max(self.n_train, 1), mode=0, G=self.Gc, gslot=gslot,
                                   n_long=self._tr_long)
            return stats
        stats, _ = ops.spmm_ce(self.rowptr, self.col, self.Zs, self.C, self.dinv, self.b[L - 1], self.y, self.mask,
                               1.0 / max(self.n_train, 1), mode=0 if train else 1, G=self.Gc if train else None,
                               gslot=self.gslot if train else None)
        return stats

    def backward(self, stats):
        L = self.L
        ms = 1.0 / (1.0 - self.p) if self.p > 0 else 1.0
        # last layer: dZs = A G (train columns only), gW_L = Hs^T dZs, gb_L from the CE statistics
        ops.spmm(self.rp_T, self.col_T, self.Gc, self.C, out=self.dZs)
        lin_bwd_weight(self.Hs[L - 2], self.dZs, self.C, K1=self.dims[L - 1], dW=self.gW[L - 1], db=self.gb_scratch)
        self.gb[L - 1].copy_(stats[4:4 + self.C])
        lin_bwd_data(self.dZs, self.W[L - 1], self.dims[L - 1], rscale=self.dinv, out1=self.dH)   # dH_{L-1}
        for l in range(L - 2, -1, -1):
            # dP_l = dH_l * [Hs_l > 0] / (1 - p), applied as the gradient rows are loaded
            lin_bwd_weight(self.AH[l], self.dH, self.dims[l + 1], K1=self.dims[l], Ym=self.Hs[l], mscale=ms,
                           dW=self.gW[l], db=self.gb[l])
            if l > 0:
                lin_bwd_data(self.dH, self.W[l], self.dims[l], Ym=self.Hs[l], mscale=ms, rscale=self.dinv,
                             out1=self.dAHs)                                   # D^-1/2 dAH_l
                ops.spmm(self.rowptr, self.col, self.dAHs, self.dims[l], rscale=self.dinv, out=self.dH)   # dH_{l-1}

    def train_body(self):
        stats = self.forward(train=True)
        self.backward(stats)
        ops.adam_(self.params, self.grads, self.m, self.v, self.lr, self.step_t)
        self.last_stats = stats
        return stats[0:1] / max(self.n_train, 1)

    @torch.no_grad()
    def evaluate(self):
        s = self.forward(train=False).cpu().numpy()
        return {"train_loss": float(s[0]) / max(self.n_train, 1),
                "train_acc": float(s[1]) / max(self.n_train, 1),
                "val_acc": float(s[2]) / max(self.n_val, 1),
                "test_acc": float(s[3]) / max(self.n_test, 1)}

    def state_tensors(self):
        return {"params": self.params, "adam_m": self.m, "adam_v": self.v, "adam_step": self.step_t}

    def load_state_tensors(self, t):
        for name, dst in (("params", self.params), ("adam_m", self.m), ("adam_v", self.v),
                          ("adam_step", self.step_t)):
            if t[name].shape != dst.shape:
                raise ValueError("checkpoint %s has shape %s, trainer %s" % (name, tuple(t[name].shape),
                                                                              tuple(dst.shape)))
            dst.copy_(t[name].to(dst.device))


class GCNInference:
    """Full-graph GCN forward in ``dtype`` (default fp16), captured into one hipGraph.

    ``weights``: [(W [in, out], b [out]), ...] (fp32, any source: a trained
    ``GCN``/``DeepGCNTrainer`` via ``from_model``, or random init)."""

    def __init__(self, g: GraphData, weights: Sequence, dtype: torch.dtype = torch.float16,
                 capture: Optional[bool] = None):
        self.dev = g.rowptr.device
        if self.dev.type == "cpu":
            dtype = torch.float32
        self.dtype = dtype
        self.ng = NormGraph.from_data(g)
        F = g.n_features
        # features pre-scaled by the column normalisation once (static input)
        self.xs = pad_cols(g.x.float() * g.dinv[:, None]).to(dtype).contiguous()
        self.W, self.b, self.Wf = [], [], []
        # gathered rows padded to whole 128-B lines (against packing to 8 elements: Reddit
        # layer 2 1.24 vs 1.40 ms, profiles/r03_cfgs) -- an aligned row touches whole lines only
        align = 64 if dtype != torch.float32 else 8
        for k, (W, b) in enumerate(weights):
            W = W.detach().float()
            if W.shape[0] < (self.xs.shape[1] if k == 0 else self.W[-1].shape[1]):
                W = torch.nn.functional.pad(
                    W, (0, 0, 0, (self.xs.shape[1] if k == 0 else self.W[-1].shape[1]) - W.shape[0]))
            out = W.shape[1]
            padded = (out + align - 1) // align * align
            Wp = torch.zeros(W.shape[0], padded)
            Wp[:, :out] = W.cpu()
            bp = torch.zeros(padded)
            bp[:out] = b.detach().float().cpu()
            self.W.append(Wp.to(self.dev, dtype).contiguous())
            self.Wf.append(Wp.to(self.dev).contiguous())        # fp32 master: lin_fwd stages it itself
            self.b.append(bp.to(self.dev).contiguous())
        self.out_dim = weights[-1][0].shape[1]
        cuda = self.dev.type == "cuda"
        # GPU: every transform on the hand-written MFMA layer (lin_fwd, fp16 / bf16 matrix
        # cores, the D^-1/2 row scale of the next gather in its epilogue) into fixed buffers
        self._lin = cuda and dtype in (torch.float16, torch.bfloat16)
        # every layer on the hand-written MFMA layer: Reddit's 602-wide first layer (a
        # weight too wide for LDS whole) takes lin_fwd's K-chunked GEMM form
        if self._lin:
            self.z = [torch.zeros(g.n, W.shape[1], dtype=dtype, device=self.dev) for W in self.Wf]
            self.dinv32 = self.ng.dinv.float().contiguous()
        self._graph = StepGraph(self._forward, warmup=2, enabled=cuda if capture is None else capture and cuda,
                                device=self.dev)

    @classmethod
    def from_model(cls, g: GraphData, model: GCN, dtype=torch.float16, capture=None):
        return cls(g, [(c.weight, c.bias) for c in model.convs], dtype, capture)

    @torch.no_grad()
    def _forward(self):
        h = self.xs
        L = len(self.W)
        for k in range(L):
            if self._lin:
                # Z = rs * (H W) on the MFMA layer; rs = D^-1/2 folded into the epilogue
                # (the input features are pre-scaled once, so layer 1 has no row scale)
                z = lin_fwd(h, self.Wf[k], None, K1=self.Wf[k].shape[0],
                            rscale=self.dinv32 if k > 0 else None, out=self.z[k])
            else:
                z = h @ self.W[k]
                if k > 0:
                    z = z * self.ng.dinv[:, None].to(z.dtype)
            h = aggregate(z, self.ng, prescaled=True, bias=self.b[k], relu=k < L - 1)
        return h

    def __call__(self) -> torch.Tensor:
        """Logits [n, out] (a view of the captured output buffer)."""
        return self._graph()[:, :self.out_dim]
