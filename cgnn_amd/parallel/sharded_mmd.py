"""Sample-sharded MMD for long sample sets (SURVEY §5 "long-context").

The reference computes the MMD of one model on one device with the full
``[2N, 2N]`` kernel matrix (Loss.py:12-32), so N is bounded by one device's
memory and time.  Here the N generated samples (and the N data samples) are
split over the ranks of a process group; rank r owns rows
``[b_r, b_r + n_r)``.

    L = (1/N²) Σ_r [ Σ_{i∈P_r} (Σ_{j∈P} k(p_i,p_j) − 2 Σ_{j∈T} k(p_i,t_j))
                     + Σ_{i∈T_r} Σ_{j∈T} k(t_i,t_j) ]

and the gradient of L w.r.t. a generated sample only needs that sample's row
(docs/KERNELS.md, "MMD gradient"):

    ∂L/∂p_i = (4/N²) (Σ_j s_j w_ij z_j − p_i Σ_j s_j w_ij),  i ∈ P_r

so each rank needs every COLUMN but only its own ROWS.  The columns are
all-gathered once (O(N·d) bytes; the O(N²·d) kernel work dominates, so an
all-gather beats a ring that would pipeline the same bytes), the HIP MMD
kernels evaluate the rank's row range against all columns (``row_begin`` /
``n_rows`` arguments of ``mmd_rbf_kernel`` and ``mmd_mfma_kernel``), and one
scalar all-reduce per model forms the loss.  The gradient stays local: no
gradient communication at all.  Parameters shared across ranks then need their
gradients SUM-reduced (the loss is one global function of all ranks' samples).

On CPU the same decomposition is evaluated densely with PyTorch (gloo tests).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import native
from ..engine.batch import MFMA_ROWS, MFMA_TILE, MMD_TILE, mmd_kernel_choice, padded_dim
from ..engine.reference import GAMMAS

# enough workgroups to fill 256 CUs several times over
_TARGET_BLOCKS = 2048


def _feature_major(x: torch.Tensor, D: int) -> torch.Tensor:
    R, N, d = x.shape
    out = torch.zeros(R, D, N, dtype=torch.float32, device=x.device)
    out[:, :d] = x.detach().float().transpose(1, 2)
    return out


def _row_partials_dense(p_loc, t_loc, P, T, chunk: int = 1024):
    """(loss partial, gradient·N²/4) of rows p_loc / t_loc against all columns
    (CPU / oracle path).  Shapes [n, d] and [N, d]; rows in chunks (memory O(chunk N))."""
    X = torch.cat([P, T], 0)
    N = P.shape[0]
    s = torch.cat([X.new_ones(N), -X.new_ones(N)])
    lw = torch.cat([X.new_ones(N), X.new_full((N,), -2.0)])
    loss = p_loc.new_zeros(())
    grads = []
    for a in range(0, p_loc.shape[0], chunk):
        pl, tl = p_loc[a:a + chunk], t_loc[a:a + chunk]
        d2 = torch.cdist(pl, X).pow(2)
        d2t = torch.cdist(tl, T).pow(2)
        E = torch.zeros_like(d2)
        W = torch.zeros_like(d2)
        for g in GAMMAS:
            e = torch.exp(-g * d2)
            E += e
            W += g * e
            loss = loss + torch.exp(-g * d2t).sum()
        loss = loss + (E * lw).sum()
        Ws = W * s
        grads.append(Ws @ X - pl * Ws.sum(1, keepdim=True))
    return loss, torch.cat(grads, 0)


def _valu_geometry(n_loc: int, N: int, R: int) -> Tuple[int, int, int]:
    rt = (n_loc + MMD_TILE - 1) // MMD_TILE
    n_tiles = 2 * ((N + MMD_TILE - 1) // MMD_TILE)
    nc = min(n_tiles, max(1, math.ceil(_TARGET_BLOCKS / (rt * R))))
    tpc = math.ceil(n_tiles / nc)
    return rt, math.ceil(n_tiles / tpc), tpc


def _mfma_geometry(n_loc: int, N: int, R: int) -> Tuple[int, int, int]:
    rb = (n_loc + MFMA_ROWS - 1) // MFMA_ROWS
    n_tiles = 2 * ((N + MFMA_TILE - 1) // MFMA_TILE)
    nc = min(n_tiles, max(1, math.ceil(_TARGET_BLOCKS / (rb * R))))
    tpc = math.ceil(n_tiles / nc)
    return rb, math.ceil(n_tiles / tpc), tpc


def row_partials(p_loc: torch.Tensor, t_loc: torch.Tensor, P: torch.Tensor, T: torch.Tensor, row_begin: int,
                 kernel: str = "auto"):
    """Loss partial ``[R]`` (un-normalised) and the gradient ``[R, n, d]`` of the
    FULL MMD w.r.t. the generated rows ``[row_begin, row_begin + n)``, given the
    gathered columns ``P``/``T`` ``[R, N, d]``.  Summing the partials of a set of
    row ranges that tile ``[0, N)`` and dividing by N² gives the MMD."""
    R, n, d = p_loc.shape
    N = P.shape[1]
    if not (0 <= row_begin and row_begin + n <= N and t_loc.shape[1] == n):
        raise ValueError("row range outside the gathered samples")
    scale = 4.0 / (N * N)
    if not p_loc.is_cuda:
        outs = [_row_partials_dense(p_loc[r].double(), t_loc[r].double(), P[r].double(), T[r].double())
                for r in range(R)]
        loss = torch.stack([o[0] for o in outs]).to(p_loc.dtype)
        grad = torch.stack([o[1] for o in outs]).to(p_loc.dtype) * scale
        return loss, grad
    hip = native.hip()
    D = padded_dim(d)
    kernel = mmd_kernel_choice(D, kernel)
    Pf, Tf = _feature_major(P, D), _feature_major(T, D)
    st = torch.cuda.current_stream(p_loc.device).cuda_stream
    dev = p_loc.device
    # true-true rows of this range (vector kernel, mode 2)
    rt, nc, tpc = _valu_geometry(n, N, R)
    lp_tt = torch.empty(R, rt * nc, dtype=torch.float32, device=dev)
    dummy = torch.empty(1, dtype=torch.float32, device=dev)
    hip.mmd(2, D, Pf.data_ptr(), Tf.data_ptr(), dummy.data_ptr(), lp_tt.data_ptr(), N, R, rt, nc, tpc, 0.0, st,
            row_begin=row_begin, n_rows=n)
    if kernel == "mfma":
        rb, nc, tpc = _mfma_geometry(n, N, R)
        gp = torch.empty(nc, R, D, n, dtype=torch.float32, device=dev)
        lp = torch.empty(R, rb * nc, dtype=torch.float32, device=dev)
        pn = (Pf * Pf).sum(1).contiguous()
        tn = (Tf * Tf).sum(1).contiguous()
        hip.mmd_mfma(0, D, Pf.data_ptr(), Tf.data_ptr(), pn.data_ptr(), tn.data_ptr(), gp.data_ptr(),
                     lp.data_ptr(), N, R, nc, tpc, scale, st, row_begin=row_begin, n_rows=n)
    else:
        gp = torch.empty(nc, R, D, n, dtype=torch.float32, device=dev)
        lp = torch.empty(R, rt * nc, dtype=torch.float32, device=dev)
        hip.mmd(0, D, Pf.data_ptr(), Tf.data_ptr(), gp.data_ptr(), lp.data_ptr(), N, R, rt, nc, tpc, scale, st,
                row_begin=row_begin, n_rows=n)
    loss = lp.sum(1) + lp_tt.sum(1)
    grad = gp.sum(0)[:, :d].transpose(1, 2)
    return loss.to(p_loc.dtype), grad.to(p_loc.dtype).contiguous()


def _gather_rows(x: torch.Tensor, counts, group) -> torch.Tensor:
    """All-gather [R, n_r, d] blocks of possibly different n_r along dim 1."""
    m = max(counts)
    pad = torch.zeros(x.shape[0], m, x.shape[2], dtype=x.dtype, device=x.device)
    pad[:, :x.shape[1]] = x
    bufs = [torch.empty_like(pad) for _ in counts]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:, :c] for b, c in zip(bufs, counts)], 1)


class _ShardedMMD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p_loc, t_loc, group, kernel):
        world = dist.get_world_size(group)
        me = dist.get_rank(group)
        cnt = torch.tensor([p_loc.shape[1]], dtype=torch.int64, device=p_loc.device)
        cnts = [torch.empty_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt, group=group)
        counts = [int(c) for c in cnts]
        P = _gather_rows(p_loc.detach(), counts, group)
        T = _gather_rows(t_loc.detach(), counts, group)
        N = P.shape[1]
        loss, grad = row_partials(p_loc.detach(), t_loc.detach(), P, T, sum(counts[:me]), kernel)
        loss = loss.contiguous()
        dist.all_reduce(loss, group=group)
        ctx.save_for_backward(grad)
        return (loss / (N * N)).to(p_loc.dtype)

    @staticmethod
    def backward(ctx, gout):
        (g,) = ctx.saved_tensors
        return gout.view(-1, 1, 1).to(g.dtype) * g, None, None, None


def mmd_loss_sharded(pred_loc: torch.Tensor, true_loc: torch.Tensor, group: Optional[object] = None,
                     kernel: str = "auto") -> torch.Tensor:
    """MMD² of the samples spread over the ranks of ``group``: each rank passes
    its shard ``[n_r, d]`` (or ``[R, n_r, d]`` for a batch of models; shards may
    differ in size) and gets the GLOBAL loss; ``backward`` fills the gradient of
    its own generated rows.  Without an initialised process group this is the
    single-device MMD."""
    batched = pred_loc.dim() == 3
    p = pred_loc if batched else pred_loc.unsqueeze(0)
    t = true_loc if batched else true_loc.unsqueeze(0)
    if p.shape != t.shape:
        raise ValueError("generated and data shards must have the same shape")
    if not (dist.is_available() and dist.is_initialized()):
        from ..ops.mmd import mmd_loss
        out = mmd_loss(p, t, kernel)
    else:
        out = _ShardedMMD.apply(p, t.detach(), group, kernel)
    return out if batched else out[0]
