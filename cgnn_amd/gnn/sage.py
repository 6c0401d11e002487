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
on the device with a stable sort -- deterministic, no atomics.  The two linear
maps of a layer are one hipBLASLt GEMM on bf16 operands (fp32 accumulation) and
the weight gradient runs split-K (``_SageLinear``).
"""
from __future__ import annotations

import math
import queue
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import native
from . import ops
from .data import GraphData


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
                 sampler: Optional[str] = None):
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
        # "device": HIP sampler on the resident CSR (default on a GPU); "host": C++/OpenMP
        self.sampler = sampler or ("device" if self.dev.type == "cuda" else "host")
        self._dsampler = None
        if self.fanouts and self.sampler == "device":
            from .sampler import DeviceSampler
            self._dsampler = DeviceSampler(g.rowptr, g.col, self.fanouts[:layers], seed)
        self.epoch = 0

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
    def _step(self, blocks, nodes_in, seeds_t):
        self.model.train()
        out = self.model(self.x[nodes_in], blocks)
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

    @torch.no_grad()
    def evaluate(self):
        """Full-graph (layer-wise exact) inference; accuracies per split."""
        self.model.eval()
        out = self.model(self.x, self.full_blocks())[:, :self.C]
        pred = out.argmax(1)
        res = {}
        for name, k in (("train_acc", 1), ("val_acc", 2), ("test_acc", 3)):
            m = self.g.mask == k
            res[name] = float((pred[m] == self.g.y[m].long()).float().mean()) if bool(m.any()) else float("nan")
        return res
