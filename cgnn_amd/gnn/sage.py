"""GraphSAGE (mean aggregator) on the HIP SpMM -- GNN track, not in the reference.

Layer:  h_i' = act( W_self h_i + W_neigh mean_{j in N(i)} h_j + b )

Two training modes:

* **full graph** -- every layer aggregates over the whole CSR (A + I) with the
  row scale 1/deg, like the GCN trainer;
* **sampled mini-batches** -- the C++ neighbour sampler (``_rt.sample_neighbors``,
  OpenMP, GIL released) draws a fan-out per layer for a batch of seed nodes and
  returns one bipartite block per layer (destination nodes are a prefix of the
  source nodes).  A background thread samples batch k+1 while the GPU trains on
  batch k.

The aggregation is the same CSR gather-sum kernel as the GCN (``spmm_kernel``);
its backward is the transposed block SpMM, for which the transposed CSR is built
on the device with a stable sort -- deterministic, no atomics.

``fused=True`` (default on a GPU; the CPU runs the same schedule through the ops'
reference branches): a hand-scheduled step on the HIP kernels only.  A layer is
``spmm`` (mean aggregate, bf16 out) + ``lin_fwd`` over the VIRTUAL concatenation
``[h_dst | agg]`` with ``[W_self; W_neigh]`` stacked (bias, ReLU, Philox dropout in
the epilogue; the first layer reads its ``h_dst`` rows straight out of the
resident feature matrix through a row index, and its gather through the global
column ids -- the batch's input features are never copied); the loss is the
fused ``spmm_ce`` over a unit-diagonal CSR (softmax cross-entropy + gradient in
one pass); the backward is ``lin_bwd_weight`` (split-K, mask-on-load) +
``lin_bwd_data`` (``dh_dst`` in fp32 straight into the ``init`` of the
transposed SpMM that scatters ``dagg``), then one RCCL all-reduce of the flat
gradient buffer and the flat Adam kernel.  ``fused=False``: PyTorch autograd
with hipBLASLt GEMMs (``_SageLinear``), the A/B baseline.
"""
from __future__ import annotations

import collections
import math
import queue
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import native
from ..utils.philox import model_key
from . import ops
from .data import GraphData
from .linear import lin_bwd_data, lin_bwd_weight, lin_fwd


def transpose_csr(rowptr: torch.Tensor, col: torch.Tensor, n_cols: int, with_perm: bool = False):
    """CSR of the transpose (rows = former columns), deterministic (stable sort);
    ``with_perm`` also returns, per transposed edge, the original edge index."""
    n_rows = rowptr.numel() - 1
    # sizes known on the host (nnz, n_cols): no device-to-host synchronisation
    rows = torch.repeat_interleave(torch.arange(n_rows, device=col.device, dtype=torch.int32),
                                   (rowptr[1:] - rowptr[:-1]).long(), output_size=col.numel())
    order = torch.sort(col.long(), stable=True).indices
    col_t = rows[order].to(torch.int32)
    counts = torch.zeros(n_cols, dtype=torch.int64, device=col.device)
    counts.index_add_(0, col.long(), torch.ones_like(col, dtype=torch.int64))
    rp_t = torch.zeros(n_cols + 1, dtype=torch.int64, device=col.device)
    rp_t[1:] = torch.cumsum(counts, 0)
    if with_perm:
        return rp_t.to(torch.int32), col_t, order.to(torch.int32)
    return rp_t.to(torch.int32), col_t


class Block:
    """One bipartite aggregation block: ``n_dst`` destination rows over ``n_src``
    source rows (the destinations are the first ``n_dst`` sources)."""

    def __init__(self, rowptr, col, n_src, device):
        self.rowptr = torch.as_tensor(np.asarray(rowptr), dtype=torch.int32).to(device)
        self.col = torch.as_tensor(np.asarray(col), dtype=torch.int32).to(device)
        self.n_dst = self.rowptr.numel() - 1
        self.n_src = int(n_src)
        deg = (self.rowptr[1:] - self.rowptr[:-1]).float()
        self.inv_deg = torch.where(deg > 0, 1.0 / deg.clamp_min(1), torch.zeros_like(deg))
        self._t = None

    def transposed(self):
        if self._t is None:
            self._t = transpose_csr(self.rowptr, self.col, self.n_src)
        return self._t


class _MeanAggregate(torch.autograd.Function):
    """agg[i] = inv_deg[i] * sum_{e in row i} h[col[e]]  (fp32, HIP SpMM on GPU)."""

    @staticmethod
    def forward(ctx, h, block: Block):
        ctx.block = block
        F = h.shape[1]
        return ops.spmm(block.rowptr, block.col, h.contiguous(), F, rscale=block.inv_deg,
                        out_dtype=torch.float32, ld_out=F)

    @staticmethod
    def backward(ctx, g):
        b = ctx.block
        rp_t, col_t = b.transposed()
        F = g.shape[1]
        # d h_j = sum_{i: j in N(i)} inv_deg[i] g_i: the row scale of the forward becomes
        # the column scale of the transposed SpMM (applied in the gather)
        return ops.spmm(rp_t, col_t, g.contiguous(), F, out_dtype=torch.float32, ld_out=F,
                        cscale=b.inv_deg), None


def mean_aggregate(h: torch.Tensor, block: Block) -> torch.Tensor:
    if h.shape[1] % 8:
        raise ValueError("feature width must be a multiple of 8 (pad the features)")
    return _MeanAggregate.apply(h, block)


class _SageLinear(torch.autograd.Function):
    """out = [h_dst | agg] @ [W_self; W_neigh] + b as ONE GEMM (K = 2F).

    On a GPU the operands are bf16 (MFMA) with fp32 accumulation and output; the
    weight gradient [h_dst | agg]^T g is a contraction over all the block's
    destination rows into a tiny [2F, out] matrix, so it runs split-K
    (``ops.tall_gemm_tn``: row chunks as one batched GEMM, fixed-order sum) -- as a
    plain GEMM it gave the whole reduction to a few dozen workgroups (the largest
    kernel of the mini-batch epoch, 341 us a call).  On the CPU everything is fp32."""

    @staticmethod
    def forward(ctx, h_dst, agg, w_self, w_neigh, b):
        lowp = h_dst.is_cuda
        dt = torch.bfloat16 if lowp else torch.float32
        X = torch.cat([h_dst.to(dt), agg.to(dt)], 1)
        W = torch.cat([w_self, w_neigh], 0).to(dt)
        out = torch.mm(X, W, out_dtype=torch.float32) if lowp else X @ W
        out += b
        ctx.save_for_backward(X, W)
        ctx.F = h_dst.shape[1]
        return out

    @staticmethod
    def backward(ctx, g):
        X, W = ctx.saved_tensors
        F = ctx.F
        lowp = X.is_cuda
        gl = g.to(X.dtype).contiguous()
        gW = ops.tall_gemm_tn(X, gl, chunk=4096)
        gX = torch.mm(gl, W.t(), out_dtype=torch.float32) if lowp else gl @ W.t()
        return gX[:, :F], gX[:, F:], gW[:F], gW[F:], g.sum(0)


class SAGE(torch.nn.Module):
    def __init__(self, in_dim: int, hidden: int, out_dim: int, layers: int = 2, dropout: float = 0.5,
                 seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        dims = [in_dim] + [hidden] * (layers - 1) + [out_dim]
        self.w_self = torch.nn.ParameterList()
        self.w_neigh = torch.nn.ParameterList()
        self.bias = torch.nn.ParameterList()
        for a, b in zip(dims[:-1], dims[1:]):
            bound = math.sqrt(6.0 / (a + b))
            self.w_self.append(torch.nn.Parameter((torch.rand(a, b, generator=g) * 2 - 1) * bound))
            self.w_neigh.append(torch.nn.Parameter((torch.rand(a, b, generator=g) * 2 - 1) * bound))
            self.bias.append(torch.nn.Parameter(torch.zeros(b)))
        self.dropout = float(dropout)

    def layer(self, k: int, h: torch.Tensor, block: Block, last: bool):
        agg = mean_aggregate(h, block)
        out = _SageLinear.apply(h[:block.n_dst], agg, self.w_self[k], self.w_neigh[k], self.bias[k])
        if not last:
            out = torch.relu(out)
            if self.training and self.dropout > 0:
                out = torch.nn.functional.dropout(out, self.dropout)
        return out

    def forward(self, x: torch.Tensor, blocks: Sequence[Block]):
        """``blocks`` ordered input layer first (the sampler's list reversed)."""
        h = x
        L = len(self.w_self)
        for k in range(L):
            h = self.layer(k, h, blocks[k], k == L - 1)
            if k < L - 1 and h.shape[1] % 8:
                h = torch.nn.functional.pad(h, (0, 8 - h.shape[1] % 8))
            if k < L - 1 and h.is_cuda:
                h = h.to(torch.bfloat16)      # the next SpMM gathers bf16 rows (fp32 sums)
        return h


class _FusedSAGE:
    """Flat-parameter GraphSAGE on the HIP kernels (see the module docstring).
    Parameters ``[W_0, b_0, ..., W_{L-1}, b_{L-1}]``, ``W_k = [W_self; W_neigh]``
    initialised exactly like :class:`SAGE` (same generator sequence)."""

    def __init__(self, x: torch.Tensor, n_features: int, hidden: int, n_classes: int, layers: int, dropout: float,
                 lr: float, seed: int, fanouts: Optional[Sequence[int]] = None):
        dev = x.device
        # the blocks' fanouts, input layer first (None: full-graph blocks); a block whose
        # fanout is at most 8 aggregates on ops.spmm_fan (rows of <= fanout picks)
        self.fan = list(reversed(list(fanouts)))[:layers] if fanouts else None
        self.dev, self.L, self.C, self.p, self.lr = dev, layers, n_classes, float(dropout), float(lr)
        F = x.shape[1]
        self.dims = [F] + [hidden] * (layers - 1) + [n_classes]
        self.ld = [(d + 7) // 8 * 8 for d in self.dims]
        self.x = x
        g = torch.Generator().manual_seed(seed)
        parts, self.offs = [], []
        off = 0
        for k, (a, b) in enumerate(zip(self.dims[:-1], self.dims[1:])):
            bound = math.sqrt(6.0 / (a + b))
            ws = (torch.rand(a, b, generator=g) * 2 - 1) * bound
            wn = (torch.rand(a, b, generator=g) * 2 - 1) * bound
            if k == 0:                       # padded feature rows stay 0 (as SAGETrainer does)
                ws[n_features:] = 0
                wn[n_features:] = 0
            parts += [torch.cat([ws, wn], 0).reshape(-1), torch.zeros(b)]
            self.offs.append((off, off + 2 * a * b, off + 2 * a * b + b))
            off += 2 * a * b + b
        self.params = torch.cat(parts).to(dev)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.W, self.b, self.gW, self.gb = [], [], [], []
        for (o0, o1, o2), a, b in zip(self.offs, self.dims[:-1], self.dims[1:]):
            self.W.append(self.params[o0:o1].view(2 * a, b))
            self.b.append(self.params[o1:o2])
            self.gW.append(self.grads[o0:o1].view(2 * a, b))
            self.gb.append(self.grads[o1:o2])
        self.keys = [model_key(seed, "sage-dropout", k) for k in range(layers)]
        self.db_scratch = torch.zeros(n_classes, dtype=torch.float32, device=dev)
        self._ident = None

    def _identity(self, n):
        """Unit-diagonal CSR, unit row scale, all-train mask of >= n rows (cached)."""
        if self._ident is None or self._ident[0].numel() < n + 1:
            m = max(n, 1024)
            ar = torch.arange(m + 1, dtype=torch.int32, device=self.dev)
            self._ident = (ar, ar[:m].clone(), torch.ones(m, dtype=torch.float32, device=self.dev),
                           torch.ones(m, dtype=torch.uint8, device=self.dev))
        rp, col, ones, tr = self._ident
        return rp[:n + 1], col[:n], ones[:n], tr[:n]

    def _step_arg(self):
        return self.step_t if self.dev.type == "cuda" else int(self.step_t.item())

    def forward(self, blocks, idx0: Optional[torch.Tensor], train: bool):
        """Layers over ``blocks`` (input layer first); ``idx0`` (int32): global ids of the
        first block's sources (None: the block's ids are global already).  Returns the
        logits [n_dst_last, ldc] and the saved per-layer tensors."""
        saved = []
        h = self.x
        step = self._step_arg()
        for k, blk in enumerate(blocks):
            F, nd = self.dims[k], blk.n_dst
            last = k == self.L - 1
            if k == 0 and idx0 is not None:
                # global source ids of the input layer's edges: the sampler's picks when it
                # kept them (idx0[local] == picks), else one gather through idx0
                gcol = getattr(blk, "gcol", None)
                col = gcol if gcol is not None else idx0[blk.col.long()]
                x1, idx1 = self.x, idx0[:nd]
            else:
                col, x1, idx1 = blk.col, h, None
            out_agg = torch.empty(nd, self.ld[k], dtype=torch.bfloat16, device=self.dev)
            # (sampled blocks only -- idx0 given; evaluation passes the full-graph blocks)
            if (idx0 is not None and self.fan is not None and self.fan[k] <= 8 and h.is_cuda
                    and h.dtype == torch.bfloat16):
                agg = ops.spmm_fan(blk.rowptr, col, h, F, self.fan[k], rscale=blk.inv_deg, out=out_agg)
            else:
                agg = ops.spmm(blk.rowptr, col, h, F, rscale=blk.inv_deg, out=out_agg)
            out = torch.empty(nd, self.ld[k + 1], dtype=torch.bfloat16, device=self.dev)
            lin_fwd(x1, self.W[k], None if last else self.b[k], x2=agg, K1=F, K2=F, relu=not last,
                    p=self.p if (train and not last) else 0.0, key=self.keys[k], step=step, idx1=idx1, n=nd, out=out)
            saved.append((x1, idx1, agg, out, blk))
            h = out
        return h, saved

    def loss_and_grad(self, logits, labels, inv_count, mask=None):
        """Fused softmax cross-entropy (+ the last bias) over the rows with mask == 1 (all
        rows by default): stats, dlogits; the last bias gradient goes straight into the
        flat gradient buffer (GPU)."""
        n = logits.shape[0]
        rp, col, ones, tr = self._identity(n)
        G = torch.empty_like(logits)
        # (GPU: the bias-gradient reduction also advances the step counter -- the
        # forward has read it for this step's dropout masks -- so Adam needs no
        # separate increment launch)
        cuda = logits.is_cuda
        stats, G = ops.spmm_ce(rp, col, logits, self.C, ones, self.b[-1], labels, tr if mask is None else mask,
                               inv_count, mode=0, G=G, db_out=self.gb[-1] if cuda else None,
                               bump=self.step_t if cuda else None)
        return stats, G

    def backward(self, saved, G, stats):
        dY = G
        ms = 1.0 / (1.0 - self.p) if self.p > 0 else 1.0
        for k in range(self.L - 1, -1, -1):
            x1, idx1, agg, out, blk = saved[k]
            F, N, nd = self.dims[k], self.dims[k + 1], blk.n_dst
            last = k == self.L - 1
            Ym, m = (None, 1.0) if last else (out, ms)
            lin_bwd_weight(x1, dY, N, x2=agg, K1=F, K2=F, Ym=Ym, mscale=m, dW=self.gW[k],
                           db=self.db_scratch if last else self.gb[k], idx1=idx1, n=nd)
            if last and not dY.is_cuda:          # (GPU: written by loss_and_grad's spmm_ce)
                self.gb[k].copy_(stats[4:4 + self.C])
            if k == 0:
                break
            dhd = torch.empty(nd, self.ld[k], dtype=torch.float32, device=self.dev)
            dagg = torch.empty(nd, self.ld[k], dtype=torch.bfloat16, device=self.dev)
            lin_bwd_data(dY, self.W[k], F, F, Ym=Ym, mscale=m, out1=dhd, out2=dagg)
            rp_t, col_t = blk.transposed()
            dY = ops.spmm(rp_t, col_t, dagg, F, cscale=blk.inv_deg, init=dhd, init_rows=nd,
                          out=torch.empty(blk.n_src, self.ld[k], dtype=torch.bfloat16, device=self.dev))

    def step(self, blocks, idx0, labels, world: int = 1, mask=None, count=None):
        """One optimisation step; returns the summed training loss (device scalar)."""
        logits, saved = self.forward(blocks, idx0, train=True)
        count = logits.shape[0] if count is None else count
        stats, G = self.loss_and_grad(logits, labels, 1.0 / (count * world), mask)
        self.backward(saved, G, stats)
        if world > 1:
            torch.distributed.all_reduce(self.grads)      # loss already scaled by 1/world: a SUM is the mean
        ops.adam_(self.params, self.grads, self.m, self.v, self.lr, self.step_t, step_done=self.params.is_cuda)
        return stats[0:1]

    def state_tensors(self):
        return {"params": self.params, "adam_m": self.m, "adam_v": self.v, "adam_step": self.step_t}

    def load_state_tensors(self, t):
        for name, dst in (("params", self.params), ("adam_m", self.m), ("adam_v", self.v),
                          ("adam_step", self.step_t)):
            if t[name].shape != dst.shape:
                raise ValueError("checkpoint %s has shape %s, trainer %s" % (name, tuple(t[name].shape),
                                                                              tuple(dst.shape)))
            dst.copy_(t[name].to(dst.device))


def _pad8(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[1]
    return x if F % 8 == 0 else torch.nn.functional.pad(x, (0, 8 - F % 8))


class SAGETrainer:
    """Node classification with GraphSAGE; ``fanouts=None`` trains on the full graph.

    Data parallel (``torch.distributed`` initialised, world > 1): every rank holds
    the whole graph (an ogbn-products CSR + features is ~1.5 GB of the 288 GB of
    HBM), the epoch's seed permutation is the same on all ranks, each global batch
    of ``batch_size * world`` seeds is split evenly, and the gradients are averaged
    by ``parallel.ddp.GradBucketer`` (bucketed RCCL all-reduce overlapped with the
    backward).  ``batch_size`` is per rank (weak scaling)."""

    def __init__(self, g: GraphData, hidden: int = 256, layers: int = 2, dropout: float = 0.5,
                 lr: float = 0.003, fanouts: Optional[List[int]] = (15, 10), batch_size: int = 1024,
                 seed: int = 0, prefetch: bool = True, standardize: bool = True, bucket_mb: float = 16.0,
                 sampler: Optional[str] = None, fused: Optional[bool] = None):
        from ..parallel import dist as pdist
        self.rank, self.world = pdist.rank(), pdist.world_size()
        self.g = g
        self.dev = g.rowptr.device
        x = g.x.float()
        if standardize:                       # column z-scores (standard preprocessing)
            x = (x - x.mean(0)) / x.std(0).clamp_min(1e-6)
        self.x = _pad8(x)
        if self.x.is_cuda:        # gathered features stored bf16 (the GEMMs take bf16 anyway)
            self.x = self.x.to(torch.bfloat16)
        self.C = g.n_classes
        F = self.x.shape[1]
        self.fused = (self.dev.type == "cuda") if fused is None else bool(fused)
        self.fanouts = list(fanouts) if fanouts else None
        self.layers = layers
        self.batch_size = int(batch_size)
        self.seed = int(seed)
        self.train_idx = torch.nonzero(g.mask.cpu() == 1).flatten().numpy()
        self._rp64 = g.rowptr.cpu().numpy().astype(np.int64)
        self._col = g.col.cpu().numpy()
        self._full = None
        self.prefetch = bool(prefetch)
        # "pipelined" (default on a GPU): the native whole-batch sampler on a side stream,
        # double-buffered; "device": the per-level HIP sampler; "host": C++/OpenMP
        self.sampler = sampler or ("pipelined" if self.dev.type == "cuda" else "host")
        self._dsampler = None
        self._psampler = None
        self._main = None
        if self.fanouts and self.sampler == "device":
            from .sampler import DeviceSampler
            self._dsampler = DeviceSampler(g.rowptr, g.col, self.fanouts[:layers], seed)
        if self.fanouts and self.sampler == "pipelined":
            from .sampler import PipelinedSampler
            self._psampler = PipelinedSampler(g.rowptr, g.col, self.fanouts[:layers], batch_size, seed)
        self.epoch = 0
        if self.fused:
            if not self.x.dtype == torch.bfloat16:
                self.x = self.x.to(torch.bfloat16)
            self.y32 = g.y.to(torch.int32)
            self._fused = _FusedSAGE(self.x, g.n_features, hidden, self.C, layers, dropout, lr, seed,
                                     fanouts=self.fanouts[:layers] if self.fanouts else None)
            self.model, self.opt, self.ddp = None, None, None
            if self.world > 1:       # identical initial parameters on every rank
                torch.distributed.broadcast(self._fused.params, 0)
            return
        # hidden width padded to a multiple of 8 (SpMM row alignment); output padded too
        self.model = SAGE(F, hidden, self.C, layers, dropout, seed).to(self.dev)
        self.model.w_self[0].data[g.n_features:] = 0
        self.model.w_neigh[0].data[g.n_features:] = 0
        self.opt = torch.optim.Adam(self.model.parameters(), lr=lr, fused=self.dev.type == "cuda")
        self.ddp = None
        if self.world > 1:
            from ..parallel.ddp import GradBucketer
            self.ddp = GradBucketer(list(self.model.parameters()), bucket_mb)
            self.ddp.broadcast_parameters(0)
        self.fanouts = list(fanouts) if fanouts else None
        self.layers = layers
        self.batch_size = int(batch_size)
        self.seed = int(seed)
        self.train_idx = torch.nonzero(g.mask.cpu() == 1).flatten().numpy()
        self._rp64 = g.rowptr.cpu().numpy().astype(np.int64)
        self._col = g.col.cpu().numpy()
        self._full = None
        self.prefetch = bool(prefetch)
        self.epoch = 0

    # ----------------------------------------------------------- checkpoint
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

    # ----------------------------------------------------------- blocks
    def full_blocks(self):
        if self._full is None:
            b = Block(self.g.rowptr.cpu().numpy(), self.g.col.cpu().numpy(), self.g.n, self.dev)
            self._full = [b] * self.layers
        return self._full

    def sample(self, seeds: np.ndarray, salt: int):
        raw = native.rt().sample_neighbors(self._rp64, self._col, seeds.astype(np.int64),
                                           list(self.fanouts[:self.layers]), self.seed * 1000003 + salt)
        return raw

    def _to_device(self, raw):
        blocks = []
        for rp, col, nodes in raw:
            blocks.append(Block(rp, col, len(nodes), self.dev))
        nodes_in = torch.as_tensor(np.asarray(raw[-1][2]), device=self.dev)
        return blocks[::-1], nodes_in

    # ----------------------------------------------------------- training
    def _step(self, blocks, nodes_in, seeds_t, labels=None, summed=False):
        """One training step; the batch's mean loss (device scalar), or with ``summed``
        (fused path) the loss summed over the batch -- no division launch per batch."""
        if self.fused:
            if labels is None:
                labels = self.y32[seeds_t.long()]
            loss = self._fused.step(blocks, nodes_in.to(torch.int32), labels, self.world)
            return loss[0] if summed else loss[0] / max(int(seeds_t.numel()), 1)
        self.model.train()
        out = self.model(self.x[nodes_in.long()], blocks)
        loss = torch.nn.functional.cross_entropy(out[:, :self.C], self.g.y[seeds_t].long())
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if self.ddp is not None:
            self.ddp.finish()
        self.opt.step()
        return loss.detach()

    def _batches(self):
        """This rank's seed batches of the epoch (the same global permutation on
        every rank; a global batch smaller than the world is dropped)."""
        rng = np.random.default_rng(self.seed + self.epoch)
        perm = rng.permutation(self.train_idx)
        gb = self.batch_size * self.world
        out = []
        for i in range(0, len(perm), gb):
            chunk = perm[i:i + gb]
            if len(chunk) < self.world:
                break
            out.append(np.array_split(chunk, self.world)[self.rank])
        return out

    def train_epoch(self):
        """One epoch; returns the mean training loss (one host sync at the end)."""
        if self.fanouts is None:
            blocks = self.full_blocks()
            if self.fused:
                n_tr = max(int((self.g.mask == 1).sum()), 1)
                loss = self._fused.step(blocks, None, self.y32, self.world, mask=self.g.mask, count=n_tr)
                self.epoch += 1
                return float(loss) / n_tr
            self.model.train()
            out = self.model(self.x, blocks)
            tr = self.g.mask == 1
            loss = torch.nn.functional.cross_entropy(out[tr][:, :self.C], self.g.y[tr].long())
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            if self.ddp is not None:
                self.ddp.finish()
            self.opt.step()
            self.epoch += 1
            return float(loss)
        batches = self._batches()
        losses = []
        if self._psampler is not None and batches:
            if self._main is None:
                self._main = torch.cuda.Stream(device=self.dev)
            # the batch loop on a stream of its own: work on the legacy default stream is
            # implicitly ordered against the sampler's stream, which serialised every
            # batch's sampling behind the previous batch's training (kernel trace, round 5)
            cur = torch.cuda.current_stream(self.dev)
            self._main.wait_stream(cur)
            with torch.cuda.stream(self._main):
                loss = self._pipelined_epoch(batches)
            cur.wait_stream(self._main)
            self.epoch += 1
            return loss
        if self._dsampler is not None:
            for k, b in enumerate(batches):
                seeds_t = torch.as_tensor(b, device=self.dev)
                blocks, nodes_in = self._dsampler.sample(seeds_t, (self.epoch * 100003 + k) * self.world + self.rank)
                losses.append(self._step(blocks, nodes_in, seeds_t))
        elif self.prefetch and len(batches) > 1:
            q: "queue.Queue" = queue.Queue(maxsize=2)

            def producer():
                for k, b in enumerate(batches):
                    q.put((b, self.sample(b, (self.epoch * 100003 + k) * self.world + self.rank)))
                q.put(None)

            th = threading.Thread(target=producer, daemon=True)
            th.start()
            while True:
                item = q.get()
                if item is None:
                    break
                seeds, raw = item
                blocks, nodes_in = self._to_device(raw)
                losses.append(self._step(blocks, nodes_in, torch.as_tensor(seeds, device=self.dev)))
            th.join()
        else:
            for k, b in enumerate(batches):
                blocks, nodes_in = self._to_device(self.sample(b, (self.epoch * 100003 + k) * self.world + self.rank))
                losses.append(self._step(blocks, nodes_in, torch.as_tensor(b, device=self.dev)))
        self.epoch += 1
        return float(torch.stack(losses).mean())

    def _pipelined_epoch(self, batches):
        ps = self._psampler
        losses = []
        # the epoch's seeds uploaded once; batch k + 1 samples on the side stream while k trains
        flat = torch.as_tensor(np.concatenate(batches).astype(np.int32), device=self.dev)
        # the epoch's labels gathered once too (fused path), not per batch
        yflat = self.y32[flat.long()] if self.fused else None
        seeds, labels, o = [], [], 0
        for b in batches:
            seeds.append(flat[o:o + len(b)])
            labels.append(yflat[o:o + len(b)] if yflat is not None else None)
            o += len(b)
        salt = lambda k: (self.epoch * 100003 + k) * self.world + self.rank
        # the seeds are valid from here on: the sampler waits for this event and for the
        # training that last read a slot, never for the whole training stream
        ready = torch.cuda.Event()
        ready.record()
        # slots - 1 batches sampled ahead: batch k + 2's sampling runs beside batch k's
        # training and is long done when the host asks for it
        depth, nb = len(ps.slots) - 1, len(batches)
        pend = collections.deque(ps.enqueue(seeds[j], salt(j), ready) for j in range(min(depth, nb)))
        for k in range(nb):
            if k + depth < nb:
                pend.append(ps.enqueue(seeds[k + depth], salt(k + depth), ready))
            cur = pend.popleft()
            blocks, nodes_in = cur.resolve()
            torch.cuda.current_stream(self.dev).wait_event(cur.slot.done)
            losses.append(self._step(blocks, nodes_in, seeds[k], labels[k], summed=self.fused))
            ps.consumed(cur)
        if self.fused:          # the per-batch means from the sums, once per epoch
            cnt = torch.tensor([max(len(b), 1) for b in batches], dtype=torch.float32)
            return float((torch.stack(losses).cpu() / cnt).mean())
        return float(torch.stack(losses).mean())

    @torch.no_grad()
    def evaluate(self):
        """Full-graph (layer-wise exact) inference; accuracies per split."""
        if self.fused:
            f = self._fused
            logits, _ = f.forward(self.full_blocks(), None, train=False)
            rp, col, ones, _ = f._identity(self.g.n)
            stats, _ = ops.spmm_ce(rp, col, logits, self.C, ones, f.b[-1], self.y32, self.g.mask, 1.0, mode=1)
            s = stats.cpu().numpy()
            cnt = [max(int((self.g.mask == k).sum()), 1) for k in (1, 2, 3)]
            return {"train_acc": float(s[1]) / cnt[0], "val_acc": float(s[2]) / cnt[1],
                    "test_acc": float(s[3]) / cnt[2]}
        self.model.eval()
        out = self.model(self.x, self.full_blocks())[:, :self.C]
        pred = out.argmax(1)
        res = {}
        for name, k in (("train_acc", 1), ("val_acc", 2), ("test_acc", 3)):
            m = self.g.mask == k
            res[name] = float((pred[m] == self.g.y[m].long()).float().mean()) if bool(m.any()) else float("nan")
        return res
