"""Differentiable MMD losses as PyTorch ops.

On a GPU tensor the fused HIP kernel computes the loss AND its gradient in
one pass (the backward only scales the saved gradient); on CPU the dense
PyTorch formula of the reference is used (Loss.py:12-32).  Both accept a
batch of independent problems ``[R, N, d]``.
"""
from __future__ import annotations

import math

import torch

from .. import native
from ..engine.batch import mmd_geometry, mmd_kernel_choice, mmd_mfma_geometry, mmd_mirror_slots, padded_dim
from ..engine.reference import GAMMAS, mmd_loss_dense


def _to_feature_major(x: torch.Tensor, D: int) -> torch.Tensor:
    R, N, d = x.shape
    out = torch.zeros(R, D, N, dtype=torch.float32, device=x.device)
    out[:, :d] = x.detach().float().transpose(1, 2)
    return out


class _MMDHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, true, kernel="auto", symmetric=True):
        hip = native.hip()
        R, N, d = pred.shape
        D = padded_dim(d)
        kernel = mmd_kernel_choice(D, kernel)
        P = _to_feature_major(pred, D)
        T = _to_feature_major(true, D)
        row_tiles, n_chunks, tpc = mmd_geometry(N, R)
        dev = pred.device
        mf_rb, mf_chunks, mf_tpc = mmd_mfma_geometry(N, R)
        mirror = mmd_mirror_slots(D, N, symmetric) if kernel == "valu" else 0
        gradp = torch.empty(max(n_chunks + mirror, mf_chunks), R, D, N, dtype=torch.float32, device=dev)
        lpart = torch.empty(R, max(row_tiles * n_chunks, mf_rb * mf_chunks), dtype=torch.float32, device=dev)
        tt = torch.zeros(R, dtype=torch.float32, device=dev)
        last = torch.zeros(R, dtype=torch.float32, device=dev)
        acc = torch.zeros(R, dtype=torch.float32, device=dev)
        step = torch.zeros(2, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        inv = 1.0 / (N * N)
        pn = (P * P).sum(1).contiguous()
        tn = (T * T).sum(1).contiguous()
        if hip.mmd_supported_d(D):          # constant true-true block
            hip.mmd(2, D, P.data_ptr(), T.data_ptr(), gradp.data_ptr(), lpart.data_ptr(), N, R,
                    row_tiles, n_chunks, tpc, 0.0, st)
            tt_parts = row_tiles * n_chunks
        else:                               # wide joints: the matrix-core kernel's mode 2
            hip.mmd_mfma(2, D, T.data_ptr(), T.data_ptr(), tn.data_ptr(), tn.data_ptr(), gradp.data_ptr(),
                         lpart.data_ptr(), N, R, mf_chunks, mf_tpc, 0.0, st)
            tt_parts = mf_rb * mf_chunks
        hip.loss_finalize(lpart.data_ptr(), tt_parts, tt.data_ptr(), last.data_ptr(),
                          acc.data_ptr(), inv, 2, 0, 0, step.data_ptr(), 0, R, st)
        if kernel == "mfma":
            hip.mmd_mfma(0, D, P.data_ptr(), T.data_ptr(), pn.data_ptr(), tn.data_ptr(), gradp.data_ptr(),
                         lpart.data_ptr(), N, R, mf_chunks, mf_tpc, 4.0 * inv, st)
            parts, chunks = mf_rb * mf_chunks, mf_chunks
        else:
            hip.mmd(0, D, P.data_ptr(), T.data_ptr(), gradp.data_ptr(), lpart.data_ptr(), N, R,
                    row_tiles, n_chunks, tpc, 4.0 * inv, st, mirror=int(mirror > 0))
            parts, chunks = row_tiles * n_chunks, n_chunks + mirror
        hip.loss_finalize(lpart.data_ptr(), parts, tt.data_ptr(), last.data_ptr(),
                          acc.data_ptr(), inv, 0, 0, 0, step.data_ptr(), 0, R, st)
        g = gradp[:chunks].sum(0)[:, :d].transpose(1, 2).contiguous()    # [R, N, d]
        ctx.save_for_backward(g)
        return last.to(pred.dtype)

    @staticmethod
    def backward(ctx, gout):
        (g,) = ctx.saved_tensors
        return (gout.view(-1, 1, 1).to(g.dtype) * g).to(gout.dtype), None, None, None


def mmd_loss(pred: torch.Tensor, true: torch.Tensor, kernel: str = "auto", symmetric: bool = True) -> torch.Tensor:
    """Biased multi-bandwidth MMD^2; ``[N,d]`` -> scalar or ``[R,N,d]`` -> ``[R]``.
    ``kernel``: 'auto' | 'mfma' (matrix cores, padded d >= 8) | 'valu'; ``symmetric``
    (vector kernel): evaluate half of the pred-pred block and mirror it."""
    batched = pred.dim() == 3
    p = pred if batched else pred.unsqueeze(0)
    t = true if batched else true.unsqueeze(0)
    if p.is_cuda:
        out = _MMDHip.apply(p, t.detach(), kernel, symmetric)
    else:
        out = torch.stack([mmd_loss_dense(p[r], t[r]) for r in range(p.shape[0])])
    return out if batched else out[0]
