"""L-layer GCN full-graph training and hipGraph-captured inference -- GNN
track, not in the reference.

``DeepGCNTrainer`` covers the depths / dtypes the fused 2-layer trainer
(``gcn.GCNTrainer``) does not: any number of layers, bf16 / fp16 / fp32
storage (BASELINE config "ogbn-arxiv 3-layer GCN full-graph bf16").  Layers are
``layers.GCNConv`` (transform, then normalised aggregation on the HIP SpMM);
optimizer is a capturable Adam; on a GPU the whole step (forward, backward,
Adam) is captured once into a hipGraph and replayed, because a graph of this
size is launch-bound (dozens of sub-100-microsecond kernels per epoch).

``GCNInference`` is the latency path (BASELINE config "Reddit 2-layer GCN fp16
single-GPU inference"): weights cast once to the inference dtype, features
pre-scaled by D^-1/2 once (the cached normalisation), bias + ReLU in the SpMM
epilogue, and the whole forward captured into one hipGraph.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from ..utils.hipgraph import StepGraph
from .data import GraphData
from .layers import GCN, NormGraph, aggregate, pad_cols


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
                 capture: Optional[bool] = None):
        self.dev = g.rowptr.device
        if self.dev.type == "cpu" and dtype != torch.float32:
            dtype = torch.float32                     # CPU reference path: fp32
        self.dtype = dtype
        self.ng = NormGraph.from_data(g)
        self.x = pad_cols(g.x.float()).to(dtype).contiguous()
        self.C = g.n_classes
        dims = [self.x.shape[1]] + [hidden] * (layers - 1) + [self.C]
        self.model = GCN(dims, dropout, seed).to(self.dev)
        with torch.no_grad():                         # padded feature rows of W1 stay 0
            self.model.convs[0].weight[g.n_features:] = 0
        cuda = self.dev.type == "cuda"
        self.opt = torch.optim.Adam(self.model.parameters(), lr=lr, capturable=cuda)
        self.idx = _splits(g)
        self.y = g.y.long()
        self.y_train = self.y[self.idx["train"]]
        self.layers = layers
        self.epoch = 0
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
        from .checkpoint import module_optimizer_tensors
        return module_optimizer_tensors(self.model, self.opt)

    def load_state_tensors(self, t):
        from .checkpoint import load_module_optimizer_tensors
        load_module_optimizer_tensors(self.model, self.opt, t)
        self._step_graph.reset()       # the optimizer state tensors were replaced


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
        self.W, self.b = [], []
        for k, (W, b) in enumerate(weights):
            W = W.detach().float()
            if k == 0 and W.shape[0] < self.xs.shape[1]:
                W = torch.nn.functional.pad(W, (0, 0, 0, self.xs.shape[1] - F))
            out = W.shape[1]
            padded = (out + 7) // 8 * 8
            Wp = torch.zeros(W.shape[0], padded)
            Wp[:, :out] = W.cpu()
            bp = torch.zeros(padded)
            bp[:out] = b.detach().float().cpu()
            self.W.append(Wp.to(self.dev, dtype).contiguous())
            self.b.append(bp.to(self.dev).contiguous())
        self.out_dim = weights[-1][0].shape[1]
        cuda = self.dev.type == "cuda"
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
            z = h @ self.W[k]
            if k > 0:
                # one elementwise pass over the narrow Z is cheaper than a per-edge
                # column-scale load in the gather (measured: 4.97 vs 5.47 ms on reddit)
                z = z * self.ng.dinv[:, None].to(z.dtype)
            h = aggregate(z, self.ng, prescaled=True, bias=self.b[k], relu=k < L - 1)
        return h

    def __call__(self) -> torch.Tensor:
        """Logits [n, out] (a view of the captured output buffer)."""
        return self._graph()[:, :self.out_dim]
