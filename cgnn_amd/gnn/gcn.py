"""Full-graph GCN training on MI355X (GNN track, not in the reference).

Model (Kipf & Welling): ``logits = Â · (dropout(relu(Â X W1 + b1)) W2) + b2``
with ``Â = D^-1/2 (A+I) D^-1/2``, softmax cross-entropy on the train split,
Adam.  Storage bf16, accumulation fp32, master weights fp32.

One epoch = one full-graph forward + backward + optimizer step:

  1. AX   = spmm(Xs)                       Xs = D^-1/2 X  (normalised once, like a cached Â)
  2. H1   = dropout(relu(AX W1 + b1))      GEMM (hipBLASLt) + fused HIP epilogue (Philox mask)
  3. Z2   = D^-1/2 (H1 W2)                 (all-gathered across ranks)
  4. loss, G = spmm_ce(Z2)                 aggregate + bias + log-softmax + NLL + dlogits, fused
  5. dY2  = D^-1/2 spmm(G)                 (G all-gathered across ranks; Â symmetric)
  6. dW2 = H1^T dY2, dH1 = dY2 W2^T, relu/dropout backward (fused), dW1 = AX^T dP1
  7. gradients all-reduced (RCCL), fused Adam

Multi-GPU: each rank owns a contiguous block of rows (1-D partition); the
static features are replicated (0.5 GB for ogbn-products, trivial against
288 GB of HBM), so layer 1 needs no communication; layer 2 needs one
all-gather of Z2 in the forward and one of G in the backward ([n, 48] bf16
each), plus one all-reduce of the ~40k gradient floats.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..parallel import dist as pdist
from ..utils.philox import model_key
from . import ops
from .data import GraphData, partition_rows


def _ru8(x):
    return (x + 7) // 8 * 8


def _mm_f32(a, b):
    """bf16 x bf16 -> fp32 output (fp32 accumulation)."""
    if a.is_cuda:
        return torch.mm(a, b, out_dtype=torch.float32)
    return a.float() @ b.float()


class GCNTrainer:
    def __init__(self, g: GraphData, hidden: int = 256, dropout: float = 0.5, lr: float = 0.01,
                 weight_decay: float = 0.0, seed: int = 0, rank: Optional[int] = None,
                 world: Optional[int] = None):
        self.rank = pdist.rank() if rank is None else rank
        self.world = pdist.world_size() if world is None else world
        self.dev = g.rowptr.device
        dev = self.dev
        self.F, self.C, self.hidden = g.n_features, g.n_classes, hidden
        self.ldx, self.ldc = _ru8(self.F), _ru8(self.C)
        self.p, self.lr, self.wd = float(dropout), float(lr), float(weight_decay)
        self.key = model_key(seed, "gcn-dropout")
        r0, r1, per, rp, col = partition_rows(g, self.rank, self.world)
        self.r0, self.r1, self.per, self.nloc = r0, r1, per, r1 - r0
        self.rowptr, self.col = rp.contiguous(), col.contiguous()
        self.dinv = g.dinv[r0:r1].contiguous()
        self.y = g.y[r0:r1].contiguous()
        self.mask = g.mask[r0:r1].contiguous()
        self.n_train = int((g.mask == 1).sum())
        self.n_val = int((g.mask == 2).sum())
        self.n_test = int((g.mask == 3).sum())
        bf = dict(dtype=torch.bfloat16, device=dev)
        # replicated normalised features Xs = D^-1/2 X, padded to ldx (zeros)
        self.Xs = torch.zeros(g.n, self.ldx, **bf)
        self.Xs[:, :self.F] = (g.x * g.dinv[:, None]).to(torch.bfloat16)
        # parameters: glorot-uniform weights, zero biases (PyG GCNConv init); one flat fp32 buffer
        gen = torch.Generator().manual_seed(seed)
        n1, n2 = self.F * hidden, hidden * self.C
        self.n_params = n1 + hidden + n2 + self.C
        flat = torch.zeros(self.n_params)
        a1 = math.sqrt(6.0 / (self.F + hidden))
        a2 = math.sqrt(6.0 / (hidden + self.C))
        flat[:n1] = (torch.rand(n1, generator=gen) * 2 - 1) * a1
        flat[n1 + hidden:n1 + hidden + n2] = (torch.rand(n2, generator=gen) * 2 - 1) * a2
        self.params = flat.to(dev)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        o = [0, n1, n1 + hidden, n1 + hidden + n2, self.n_params]
        self.W1 = self.params[o[0]:o[1]].view(self.F, hidden)
        self.b1 = self.params[o[1]:o[2]]
        self.W2 = self.params[o[2]:o[3]].view(hidden, self.C)
        self.b2 = self.params[o[3]:o[4]]
        self.gW1 = self.grads[o[0]:o[1]].view(self.F, hidden)
        self.gb1 = self.grads[o[1]:o[2]]
        self.gW2 = self.grads[o[2]:o[3]].view(hidden, self.C)
        self.gb2 = self.grads[o[3]:o[4]]
        # activations / workspaces (rows of this rank; Z2/G padded to `per` rows for all-gather)
        n = self.nloc
        self.AX = torch.zeros(n, self.ldx, **bf)
        self.H1 = torch.zeros(n, hidden, **bf)
        self.dH1 = torch.zeros(n, hidden, **bf)
        self.W2b = torch.zeros(hidden, self.ldc, **bf)
        self.Z2loc = torch.zeros(per, self.ldc, **bf)
        self.Gloc = torch.zeros(per, self.ldc, **bf)
        self.dY2 = torch.zeros(n, self.ldc, **bf)
        if self.world > 1:
            self.Z2 = torch.zeros(per * self.world, self.ldc, **bf)
            self.G = torch.zeros(per * self.world, self.ldc, **bf)
        else:
            self.Z2, self.G = self.Z2loc, self.Gloc
        self.epoch = 0
        self.last_stats = None

    # ------------------------------------------------------------------ passes
    def _all_gather(self, out, inp):
        if self.world > 1:
            torch.distributed.all_gather_into_tensor(out, inp)

    def forward(self, train: bool):
        n, F, C = self.nloc, self.F, self.C
        ops.spmm(self.rowptr, self.col, self.Xs, F, rscale=self.dinv, out=self.AX)
        W1b = self.W1.to(torch.bfloat16)
        if self.AX.is_cuda:
            torch.mm(self.AX[:, :F], W1b, out=self.H1)
        else:
            self.H1.copy_((self.AX[:, :F].float() @ W1b.float()).to(torch.bfloat16))
        ops.bias_relu_dropout_(self.H1, self.b1, self.hidden, self.p if train else 0.0, self.key, self.epoch)
        self.W2b[:, :C] = self.W2.to(torch.bfloat16)
        y2 = _mm_f32(self.H1, self.W2b)
        torch.mul(y2, self.dinv[:, None], out=y2)
        self.Z2loc[:n] = y2.to(torch.bfloat16)
        self._all_gather(self.Z2, self.Z2loc)
        stats, _ = ops.spmm_ce(self.rowptr, self.col, self.Z2, C, self.dinv, self.b2, self.y, self.mask,
                               1.0 / max(self.n_train, 1), mode=0 if train else 1,
                               G=self.Gloc[:n] if train else None)
        return stats

    def backward(self, stats):
        n, F, C = self.nloc, self.F, self.C
        self._all_gather(self.G, self.Gloc)
        ops.spmm(self.rowptr, self.col, self.G, C, rscale=self.dinv, out=self.dY2)
        dY2 = self.dY2[:, :C]
        self.gW2.copy_(_mm_f32(self.H1.t(), dY2))
        self.gb2.copy_(stats[4:4 + C])
        if self.dH1.is_cuda:
            torch.mm(dY2, self.W2b[:, :C].t(), out=self.dH1)
        else:
            self.dH1.copy_((dY2.float() @ self.W2b[:, :C].float().t()).to(torch.bfloat16))
        ops.relu_dropout_bwd_(self.dH1, self.H1, self.p)
        self.gW1.copy_(_mm_f32(self.AX[:, :F].t(), self.dH1))
        torch.sum(self.dH1, 0, dtype=torch.float32, out=self.gb1)
        if self.world > 1:
            torch.distributed.all_reduce(self.grads)

    def train_step(self):
        stats = self.forward(train=True)
        self.backward(stats)
        ops.adam_(self.params, self.grads, self.m, self.v, self.lr, self.step_t, wd=self.wd)
        self.last_stats = stats
        self.epoch += 1
        return stats

    @torch.no_grad()
    def evaluate(self):
        """Accuracies on train / valid / test (no dropout), reduced over ranks."""
        stats = self.forward(train=False).clone()
        if self.world > 1:
            torch.distributed.all_reduce(stats)
        s = stats.cpu().numpy()
        return {"train_loss": float(s[0]) / max(self.n_train, 1),
                "train_acc": float(s[1]) / max(self.n_train, 1),
                "val_acc": float(s[2]) / max(self.n_val, 1),
                "test_acc": float(s[3]) / max(self.n_test, 1)}

    def train_loss(self):
        s = self.last_stats.clone()
        if self.world > 1:
            torch.distributed.all_reduce(s)
        return float(s[0]) / max(self.n_train, 1)


def smoke_step():
    """One tiny GCN training step on cuda:0 (used by __graft_entry__.smoke)."""
    from .data import synthetic
    g = synthetic("cora", seed=0, device="cuda:0")
    tr = GCNTrainer(g, hidden=64, rank=0, world=1)
    tr.train_step()
    tr.train_step()
    res = tr.evaluate()
    torch.cuda.synchronize()
    assert math.isfinite(res["train_loss"]), res
    return res
