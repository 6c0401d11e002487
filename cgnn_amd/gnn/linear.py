"""Fused dense layers of the GNN track (``csrc/kernels/gnn_linear.hip``).

Three ops cover the dense half of every message-passing layer (GraphSAGE, the GAT
projection, each layer of the L-layer GCN), bf16 storage / fp32 accumulation:

* :func:`lin_fwd`         ``Y = epi([X1 | X2] W + b)``, epi = ReLU, Philox dropout
                          (the fused-kernel mask convention, keyed by global row and
                          a device step counter), row scale;
* :func:`lin_bwd_data`    ``[dX1 | dX2] = rs * ((dY * m) W^T)``;
* :func:`lin_bwd_weight`  ``dW, db = [X1 | X2]^T (dY * m), colsum(dY * m)``.

``m = [Ym > 0] / (1 - p)``: the mask is recovered from the layer's stored output
``Ym`` (after ReLU and dropout), so no mask tensor exists.  ``[X1 | X2]`` is a
virtual concatenation (no copy).  Every op has a CPU branch that is the fp32
reference of the same arithmetic (operands rounded to bf16 as the kernels see
them) -- the numerics oracle of the GPU tests.  On a GPU the HIP kernels are
mandatory: a shape no compiled variant covers raises.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import native
from ..utils import checks
from .ops import _st, _step_args, _step_value, dropout_keep_mask

_GPART = {}
_WIMG = {}


def _wimg(dev, nbytes):
    """Scratch for the bf16 LDS image of a weight (written by the launcher each call;
    cached per device and size, so a captured hipGraph keeps its address)."""
    if nbytes < 0:
        raise RuntimeError("no HIP variant for this weight shape")
    key = (dev.index, int(nbytes))
    buf = _WIMG.get(key)
    if buf is None:
        buf = _WIMG[key] = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    return buf


def _ptr(t):
    return t.data_ptr() if t is not None else 0


def _check(rc, what):
    if rc != 0:
        raise RuntimeError("%s: no HIP variant / bad shape (code %d)" % (what, rc))


def _bf(t):
    return t.to(torch.bfloat16).float()


def _cat(x1, K1, x2, K2):
    a = x1[:, :K1].float()
    return a if x2 is None else torch.cat([a, x2[:, :K2].float()], 1)


def lin_fwd(x1: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None, x2: Optional[torch.Tensor] = None,
            K1: Optional[int] = None, K2: Optional[int] = None, relu: bool = False, p: float = 0.0, key=(0, 0),
            step=0, row0: int = 0, rscale: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
            ldy: Optional[int] = None, idx1: Optional[torch.Tensor] = None, n: Optional[int] = None,
            tail: Optional[torch.Tensor] = None, nsplit: Optional[int] = None, tk: int = 1) -> torch.Tensor:
    """``out[:, :N] = epi([x1[:, :K1] | x2[:, :K2]] @ W + bias)`` in bf16 (columns N..ldy zero);
    fp16 operands (``x1`` fp16, GPU) run the same kernel on the fp16 matrix cores (the
    inference path: no dropout, no fp32 tail).

    ``W``: fp32 [K1 + K2, N]; ``step``: int or device int32[1] (read at launch time);
    ``idx1`` (int32): row r reads ``x1[idx1[r]]`` (gather-on-load); ``n``: output rows
    (default ``len(idx1)`` or the rows of x2 / x1).
    ``tail`` (fp32, with ``nsplit``): the columns ``c >= nsplit`` are written exactly, as
    planes of ``tk`` columns -- ``tail[(c - nsplit) // tk, row, (c - nsplit) % tk]`` --
    instead of bf16 into ``out`` (whose columns then stop at ``nsplit``)."""
    if n is None:
        n = idx1.shape[0] if idx1 is not None else (x2.shape[0] if x2 is not None else x1.shape[0])
    K1 = x1.shape[1] if K1 is None else int(K1)
    K2 = 0 if x2 is None else (x2.shape[1] if K2 is None else int(K2))
    N = W.shape[1]
    if W.shape[0] != K1 + K2:
        raise ValueError("W has %d rows, inputs give K = %d" % (W.shape[0], K1 + K2))
    if tail is not None:
        if nsplit is None or nsplit % 4 or (N - nsplit) % tk or tail.numel() < (N - nsplit) * n:
            raise ValueError("lin_fwd tail: nsplit %% 4 == 0 and [%d, n, %d] fp32 planes needed" % ((N - nsplit) // tk, tk))
    et = 1 if x1.dtype == torch.float16 else 0        # fp16 storage: the inference path
    if out is None:
        ldy = ldy or ((N if tail is None else nsplit) + 7) // 8 * 8
        out = torch.empty(n, ldy, dtype=torch.float16 if et else torch.bfloat16, device=x1.device)
    if checks.enabled():
        checks.index(idx1, x1.shape[0], "lin_fwd idx1")
        if idx1 is None:
            checks.rows(x1, n, "lin_fwd x1")
        checks.rows(x2, n if x2 is not None else 0, "lin_fwd x2")
        checks.rows(out, n, "lin_fwd out")
        checks.rows(rscale, n if rscale is not None else 0, "lin_fwd rscale")
    if x1.is_cuda:
        sv, sp = _step_args(step)
        hip = native.hip()
        img = _wimg(x1.device, hip.gnn_lin_fwd_image_bytes(K1 + K2, N, out.stride(0)))
        rc = hip.gnn_lin_fwd(x1.data_ptr(), x1.stride(0), K1, _ptr(x2), x2.stride(0) if x2 is not None else 0,
                                      K2, W.data_ptr(), N, _ptr(bias), out.data_ptr(), out.stride(0), n, int(relu),
                                      float(p), int(key[0]), int(key[1]), sv, int(row0), sp, _ptr(rscale), _st(x1),
                                      idx1=_ptr(idx1), wimg=img.data_ptr(), yf=_ptr(tail),
                                      nsplit=int(nsplit or 0), tk=int(tk), et=et)
        _check(rc, "lin_fwd")
        return out
    a = x1[idx1.long()] if idx1 is not None else x1[:n]
    y = _cat(a, K1, None if x2 is None else x2[:n], K2) @ _bf(W)
    if bias is not None:
        y = y + bias.float()
    if relu:
        y = torch.relu(y)
    if p > 0:
        keep = dropout_keep_mask(n, N, p, key, _step_value(step), row0)
        y = torch.where(keep, y / (1 - p), torch.zeros_like(y))
    if rscale is not None:
        y = y * rscale[:, None].float()
    out[:n].zero_()
    if tail is not None:
        out[:n, :nsplit] = y[:, :nsplit].to(torch.bfloat16)
        P = (N - nsplit) // tk
        tail.view(-1)[:P * n * tk].view(P, n, tk).copy_(y[:, nsplit:].reshape(n, P, tk).transpose(0, 1))
        return out
    out[:n, :N] = y.to(torch.bfloat16)
    return out


def _masked(dY, N, Ym, mscale):
    g = dY[:, :N].float()
    if Ym is not None:
        g = torch.where(Ym[:, :N].float() > 0, g, torch.zeros_like(g))
    return _bf(g * mscale) if (Ym is not None or mscale != 1.0) else g


def lin_bwd_data(dY: torch.Tensor, W: torch.Tensor, K1: int, K2: int = 0, Ym: Optional[torch.Tensor] = None,
                 mscale: float = 1.0, rscale: Optional[torch.Tensor] = None, out1: Optional[torch.Tensor] = None,
                 out2: Optional[torch.Tensor] = None):
    """``[out1 | out2] = rscale * ((dY[:, :N] * m) @ W^T)``, ``m = [Ym > 0] * mscale``; bf16
    (``out1`` may be fp32).  Returns (out1, out2) (out2 None when K2 == 0)."""
    n, N = dY.shape[0], W.shape[1]
    if out1 is None:
        out1 = torch.empty(n, (K1 + 7) // 8 * 8, dtype=torch.bfloat16, device=dY.device)
    if K2 and out2 is None:
        out2 = torch.empty(n, (K2 + 7) // 8 * 8, dtype=torch.bfloat16, device=dY.device)
    if dY.is_cuda:
        hip = native.hip()
        img = _wimg(dY.device, hip.gnn_lin_bwd_image_bytes(int(K1) + int(K2), N))
        rc = hip.gnn_lin_bwd_data(dY.data_ptr(), dY.stride(0), _ptr(Ym), Ym.stride(0) if Ym is not None else 0,
                                           float(mscale), N, W.data_ptr(), int(K1), int(K2), out1.data_ptr(),
                                           out1.stride(0), _ptr(out2) if K2 else 0,
                                           out2.stride(0) if K2 else 0, _ptr(rscale), n, _st(dY),
                                           dx1_f32=int(out1.dtype == torch.float32), wimg=img.data_ptr())
        _check(rc, "lin_bwd_data")
        return out1, (out2 if K2 else None)
    d = _masked(dY, N, Ym, mscale) @ _bf(W).t()
    if rscale is not None:
        d = d * rscale[:, None].float()
    out1[:n, :K1] = d[:, :K1].to(out1.dtype)
    if K2:
        out2[:, :K2] = d[:, K1:].to(torch.bfloat16)
    return out1, (out2 if K2 else None)


def lin_bwd_weight(x1: torch.Tensor, dY: torch.Tensor, N: int, x2: Optional[torch.Tensor] = None,
                   K1: Optional[int] = None, K2: Optional[int] = None, Ym: Optional[torch.Tensor] = None,
                   mscale: float = 1.0, dW: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None,
                   idx1: Optional[torch.Tensor] = None, n: Optional[int] = None):
    """``dW = [x1 | x2]^T (dY * m)`` (fp32 [K1 + K2, N]) and ``db = colsum(dY * m)`` (fp32 [N]);
    split-K over row chunks, fixed-order reduction (deterministic).  ``idx1`` / ``n`` as in
    :func:`lin_fwd` (rows of dY by default)."""
    if n is None:
        n = dY.shape[0]
    K1 = x1.shape[1] if K1 is None else int(K1)
    K2 = 0 if x2 is None else (x2.shape[1] if K2 is None else int(K2))
    dev = x1.device
    if dW is None:
        dW = torch.empty(K1 + K2, N, dtype=torch.float32, device=dev)
    if db is None:
        db = torch.empty(N, dtype=torch.float32, device=dev)
    if checks.enabled():
        checks.index(idx1, x1.shape[0], "lin_bwd_weight idx1")
        checks.rows(dY, n, "lin_bwd_weight dY")
    if x1.is_cuda:
        hip = native.hip()
        chunks = hip.gnn_lin_wgrad_chunks(max(n, 1), N, K1 + K2)
        shape = (chunks, K1 + K2 + 1, N)
        key = (dev.index, shape)
        gp = _GPART.get(key)
        if gp is None:
            gp = _GPART[key] = torch.empty(shape, dtype=torch.float32, device=dev)
        rc = hip.gnn_lin_bwd_weight(x1.data_ptr(), x1.stride(0), K1, _ptr(x2), x2.stride(0) if x2 is not None else 0,
                                    K2, dY.data_ptr(), dY.stride(0), _ptr(Ym), Ym.stride(0) if Ym is not None else 0,
                                    float(mscale), N, gp.data_ptr(), dW.data_ptr(), db.data_ptr(), n, _st(x1),
                                    idx1=_ptr(idx1))
        _check(rc, "lin_bwd_weight")
        return dW, db
    g = _masked(dY[:n], N, None if Ym is None else Ym[:n], mscale)
    a = x1[idx1.long()] if idx1 is not None else x1[:n]
    dW.copy_(_cat(a, K1, None if x2 is None else x2[:n], K2).t() @ g)
    db.copy_(g.sum(0))
    return dW, db
