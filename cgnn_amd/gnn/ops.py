"""GNN-track device ops (HIP on GPU tensors, PyTorch reference on CPU tensors).

The CPU branch is the numerical reference used by the tests (and lets the
models run in CI); on a GPU the HIP kernels of csrc/kernels/gnn_sparse.hip are
mandatory -- a missing extension raises instead of silently falling back.
"""
from __future__ import annotations

import torch

from .. import native
from ..utils import philox


def _st(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _row_ids(rowptr):
    n = rowptr.numel() - 1
    counts = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    return torch.repeat_interleave(torch.arange(n, device=rowptr.device), counts)


def spmm(rowptr, col, X, F, rscale=None, bias=None, relu=False, out=None, out_dtype=torch.bfloat16,
         ld_out=None):
    """Y[i,:F] = act(rscale[i] * sum_{j in N(i)} X[j,:F] + bias); X is [*, ldx]."""
    n = rowptr.numel() - 1
    ldo = ld_out or X.shape[1]
    if out is None:
        out = torch.empty(n, ldo, dtype=out_dtype, device=X.device)
    if X.is_cuda:
        hip = native.hip()
        hip.gnn_spmm(rowptr.data_ptr(), col.data_ptr(), X.data_ptr(), out.data_ptr(),
                     rscale.data_ptr() if rscale is not None else 0,
                     bias.data_ptr() if bias is not None else 0, n, F, X.shape[1], out.shape[1],
                     int(X.dtype == torch.bfloat16), int(out.dtype == torch.bfloat16), int(relu), _st(X))
        return out
    rows = _row_ids(rowptr)
    acc = torch.zeros(n, F, dtype=torch.float32)
    acc.index_add_(0, rows, X[col.long(), :F].float())
    if rscale is not None:
        acc = acc * rscale[:, None]
    if bias is not None:
        acc = acc + bias[:F]
    if relu:
        acc = acc.clamp_min(0)
    out.zero_()
    out[:, :F] = acc.to(out.dtype)
    return out


def spmm_ce(rowptr, col, Z, C, rscale, bias, labels, mask, inv_count, mode=0, G=None):
    """Layer-2 aggregate + log-softmax + NLL.  Returns (stats[68] summed, G)."""
    n = rowptr.numel() - 1
    ld = Z.shape[1]
    if Z.is_cuda:
        hip = native.hip()
        nb = hip.gnn_spmm_ce_blocks(n)
        stats = torch.empty(nb, 68, dtype=torch.float32, device=Z.device)
        if G is None and mode == 0:
            G = torch.empty(n, ld, dtype=torch.bfloat16, device=Z.device)
        hip.gnn_spmm_ce(rowptr.data_ptr(), col.data_ptr(), Z.data_ptr(), rscale.data_ptr(), bias.data_ptr(),
                        labels.data_ptr(), mask.data_ptr(), stats.data_ptr(), G.data_ptr() if G is not None else 0,
                        0, n, C, ld, mode, float(inv_count), _st(Z))
        return stats.sum(0), G
    rows = _row_ids(rowptr)
    acc = torch.zeros(n, C, dtype=torch.float32)
    acc.index_add_(0, rows, Z[col.long(), :C].float())
    logits = acc * rscale[:, None] + bias[:C]
    lsm = torch.log_softmax(logits, 1)
    y = labels.long()
    tr = mask == 1
    stats = torch.zeros(68)
    stats[0] = -(lsm[tr, y[tr]]).sum()
    pred = logits.argmax(1)
    for k in (1, 2, 3):
        stats[k] = ((pred == y) & (mask == k)).sum().float()
    dl = torch.softmax(logits, 1)
    dl[torch.arange(n), y] -= 1
    dl = dl * (tr[:, None].float() * inv_count)
    stats[4:4 + C] = dl.sum(0)
    if mode == 0:
        if G is None:
            G = torch.zeros(n, ld, dtype=Z.dtype)
        G.zero_()
        G[:, :C] = (dl * rscale[:, None]).to(G.dtype)
    return stats, G


def bias_relu_dropout_(H, bias, F, p, key, step):
    """In place: H = dropout(relu(H + bias)) (Philox mask keyed by (row, col/4, step))."""
    if H.is_cuda:
        native.hip().gnn_bias_relu_dropout(H.data_ptr(), bias.data_ptr(), H.shape[0], F, H.shape[1],
                                           float(p), int(key[0]), int(key[1]), int(step), _st(H))
        return H
    import numpy as np
    x = torch.relu(H[:, :F].float() + bias[:F])
    if p > 0:
        rows = np.arange(H.shape[0], dtype=np.uint32)[:, None]
        cols = np.arange(F)
        words = philox.philox4x32_10(rows, (cols // 4).astype(np.uint32)[None, :], step,
                                     philox.RNG_DROPOUT, key[0], key[1])
        w = np.stack(words, -1)                       # [n, F, 4]
        r = np.take_along_axis(w, (cols % 4)[None, :, None].repeat(H.shape[0], 0), -1)[..., 0]
        keep = torch.from_numpy(r.astype(np.uint64) >= np.uint64(int(p * 4294967296.0)))
        x = torch.where(keep, x / (1 - p), torch.zeros_like(x))
    H.zero_()
    H[:, :F] = x.to(H.dtype)
    return H


def relu_dropout_bwd_(dH, H, p):
    if dH.is_cuda:
        native.hip().gnn_relu_dropout_bwd(dH.data_ptr(), H.data_ptr(), dH.numel(), float(p), _st(dH))
        return dH
    dH.copy_(torch.where(H.float() > 0, dH.float() / (1 - p), torch.zeros_like(dH, dtype=torch.float32)).to(dH.dtype))
    return dH


def adam_(param, grad, m, v, lr, step_t, b1=0.9, b2=0.999, eps=1e-8, wd=0.0):
    """PyTorch-semantics Adam on flat fp32 buffers; ``step_t`` is a device int32[1]
    holding the number of completed steps (incremented here)."""
    if param.is_cuda:
        native.hip().gnn_adam(param.data_ptr(), m.data_ptr(), v.data_ptr(), grad.data_ptr(), param.numel(),
                              float(lr), float(b1), float(b2), float(eps), float(wd), step_t.data_ptr(),
                              _st(param))
        step_t.add_(1)
        return param
    t = float(step_t.item()) + 1
    m.mul_(b1).add_(grad, alpha=1 - b1)
    v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
    mh = m / (1 - b1 ** t)
    vh = v / (1 - b2 ** t)
    param.sub_(lr * (mh / (vh.sqrt() + eps) + wd * param))
    step_t.add_(1)
    return param
