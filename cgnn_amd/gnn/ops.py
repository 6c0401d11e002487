"""GNN-track device ops (HIP on GPU tensors, PyTorch reference on CPU tensors).

The CPU branch is the numerical reference used by the tests (and lets the
models run in CI); on a GPU the HIP kernels of csrc/kernels/gnn_sparse.hip are
mandatory -- a missing extension raises instead of silently falling back.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import native
from ..utils import checks, philox


def _st(t):
    # the raw pointer of the device's current stream, without building a torch Stream
    # object per launch (several us of host time; ~20 launches per SAGE mini-batch)
    return torch._C._cuda_getCurrentRawStream(t.get_device())


def _row_ids(rowptr):
    n = rowptr.numel() - 1
    counts = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    return torch.repeat_interleave(torch.arange(n, device=rowptr.device), counts)


_DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def dtype_code(dt) -> int:
    """Element-type code of the sparse kernels (0 fp32, 1 bf16, 2 fp16)."""
    if dt not in _DT_CODE:
        raise TypeError("sparse kernels take fp32 / bf16 / fp16, got %s" % dt)
    return _DT_CODE[dt]


def spmm(rowptr, col, X, F, rscale=None, bias=None, relu=False, out=None, out_dtype=torch.bfloat16,
         ld_out=None, unit_col=-1, init=None, cscale=None, init_rows=None, short_rows=None):
    """Y[i,:F] = act(rscale[i] * (init[i] + sum_{j in N(i)} cscale[j] X[j,:F]) + bias); X is [*, ldx].
    Padding columns of Y are written 0, except ``unit_col`` which is written 1
    (a ones column that turns the bias gradient into one more GEMM row).
    ``init`` (optional fp32 [init_rows, >=F], default all n rows): partial sums of other
    edges (split aggregation) added to the first ``init_rows`` rows.
    ``cscale`` (optional fp32 per source row): a column scale applied in the gather.
    Rows wider than 512 columns run as 512-column slabs (one launch each); narrower
    slabs were measured slower (round 4, profiles/r04_spmm).
    ``short_rows`` (default: at most 2 entries per row on average, from ``col``'s
    length): the kernel that gives each sub-group 4 consecutive rows (a transposed
    sampled block); bit-identical to the one-row-per-sub-group kernel."""
    n = rowptr.numel() - 1
    if short_rows is None:
        short_rows = col.numel() <= 2 * n
    ldo = ld_out or X.shape[1]
    if out is None:
        out = torch.empty(n, ldo, dtype=out_dtype, device=X.device)
    if checks.enabled():
        checks.csr(rowptr, col, X.shape[0], "spmm")
        checks.rows(out, n, "spmm out")
        checks.rows(rscale, n, "spmm rscale")
        checks.rows(cscale, X.shape[0], "spmm cscale")
    if X.is_cuda:
        hip = native.hip()
        hip.gnn_spmm(rowptr.data_ptr(), col.data_ptr(), X.data_ptr(), out.data_ptr(),
                     rscale.data_ptr() if rscale is not None else 0,
                     bias.data_ptr() if bias is not None else 0, n, F, X.shape[1], out.shape[1],
                     dtype_code(X.dtype), dtype_code(out.dtype), int(relu), int(unit_col),
                     _st(X), init.data_ptr() if init is not None else 0,
                     init.stride(0) if init is not None else 0,
                     cscale.data_ptr() if cscale is not None else 0,
                     -1 if init_rows is None else int(init_rows), int(bool(short_rows)))
        return out
    rows = _row_ids(rowptr)
    acc = torch.zeros(n, F, dtype=torch.float32)
    src = X[col.long(), :F].float()
    if cscale is not None:
        src = src * cscale[col.long()][:, None]
    acc.index_add_(0, rows, src)
    if init is not None:
        r = n if init_rows is None else int(init_rows)
        acc[:r] = acc[:r] + init[:r, :F].float()
    if rscale is not None:
        acc = acc * rscale[:, None]
    if bias is not None:
        acc = acc + bias[:F]
    if relu:
        acc = acc.clamp_min(0)
    out[:n].zero_()
    out[:n, :F] = acc.to(out.dtype)
    if unit_col >= 0:
        out[:n, unit_col] = 1
    return out


def spmm_fan(rowptr, col, X, F, max_deg, rscale=None, out=None):
    """``spmm`` (bf16, no bias / init / column scale) for rows of at most ``max_deg``
    entries -- a sampled block whose fanout bounds every row: at most 8, a pipelined
    persistent kernel (gnn_sparse.hip, spmm_fan_pipe_kernel); same sums, bit for bit."""
    n = rowptr.numel() - 1
    if out is None:
        out = torch.empty(n, X.shape[1], dtype=torch.bfloat16, device=X.device)
    if not X.is_cuda:
        return spmm(rowptr, col, X, F, rscale=rscale, out=out)
    if X.dtype != torch.bfloat16 or out.dtype != torch.bfloat16:
        raise TypeError("spmm_fan: bf16 in and out")
    if checks.enabled():
        checks.csr(rowptr, col, X.shape[0], "spmm_fan")
        checks.rows(out, n, "spmm_fan out")
        checks.rows(rscale, n, "spmm_fan rscale")
        if n > 0 and int((rowptr[1:] - rowptr[:-1]).max()) > max_deg:
            raise ValueError("spmm_fan: a row has more than max_deg = %d entries" % max_deg)
    native.hip().gnn_spmm_fan(rowptr.data_ptr(), col.data_ptr(), X.data_ptr(), out.data_ptr(),
                              rscale.data_ptr() if rscale is not None else 0, n, F, X.shape[1], out.shape[1],
                              X.shape[0], col.numel(), int(max_deg), _st(X))
    return out


_DB_INDEX = {}


class EllImage:
    """ELL image of a CSR for ``spmm_ell``.  ``ell``: int32 [n, 8], the row's column ids
    (-1 past its end), or {-2, e0, e1, -1...} for a row of more than 8 entries (its CSR
    range); ``long_rows``: int32 [n_long], the ids of those rows, ascending (the GPU
    sums them in a launch of their own, so the short-row loop has no data-dependent
    inner loop)."""
    __slots__ = ("ell", "long_rows", "n_long")

    def __init__(self, ell, long_rows):
        self.ell, self.long_rows, self.n_long = ell, long_rows, int(long_rows.numel())

    @property
    def n(self):
        return self.ell.shape[0]


def ell_image(rowptr, col):
    """:class:`EllImage` of the CSR (rowptr, col), built once at setup."""
    n = rowptr.numel() - 1
    ell = torch.empty(n, 8, dtype=torch.int32, device=col.device)
    rp = rowptr.long()
    deg = rp[1:] - rp[:-1]
    long_rows = torch.nonzero(deg > 8).flatten().to(torch.int32).contiguous()
    if col.is_cuda:
        native.hip().gnn_ell_build(rowptr.data_ptr(), col.data_ptr(), ell.data_ptr(), n, _st(col))
        return EllImage(ell, long_rows)
    ell.fill_(-1)
    for u in range(8):
        has = deg > u
        ell[has, u] = col[(rp[:-1] + u)[has]]
    longr = deg > 8
    ell[longr] = -1
    ell[longr, 0] = -2
    ell[longr, 1] = rp[:-1][longr].to(torch.int32)
    ell[longr, 2] = rp[1:][longr].to(torch.int32)
    return EllImage(ell, long_rows)


def spmm_ell(img, col, X, F, rscale=None, out=None):
    """Y[i,:F] = rscale[i] * sum_{j in N(i)} X[j,:F] from an :class:`EllImage` (bf16,
    F <= 64; the same sums as ``spmm`` over the CSR the image was built from)."""
    ell = img.ell
    n = ell.shape[0]
    if out is None:
        out = torch.empty(n, X.shape[1], dtype=torch.bfloat16, device=X.device)
    if X.is_cuda:
        native.hip().gnn_spmm_ell(ell.data_ptr(), col.data_ptr(), X.data_ptr(), out.data_ptr(),
                                  rscale.data_ptr() if rscale is not None else 0, n, F, X.shape[1],
                                  out.shape[1], X.shape[0], img.long_rows.data_ptr(), img.n_long, _st(X))
        return out
    acc = torch.zeros(n, F, dtype=torch.float32)
    short = ell[:, 0] != -2                    # a long row's slots hold its CSR range
    for u in range(8):
        j = ell[:, u].long()
        ok = (j >= 0) & short
        acc[ok] += X[j[ok], :F].float()
    longr = (~short).nonzero().flatten()
    for i in longr.tolist():
        e0, e1 = int(ell[i, 1]), int(ell[i, 2])
        acc[i] = X[col[e0:e1].long(), :F].float().sum(0)
    if rscale is not None:
        acc = acc * rscale[:, None]
    out[:n].zero_()
    out[:n, :F] = acc.to(out.dtype)
    return out


CE_LONG_DEGREE = 256     # rows above this degree get a wave of their own in spmm_ce


def long_row_order(deg: torch.Tensor, threshold: Optional[int] = None):
    """Row order for ``spmm_ce(..., n_long=k)``: the rows of degree > threshold first (in
    their original order), then the others; returns (order, k).  Default threshold
    CE_LONG_DEGREE; 0 disables the long-row mode."""
    if threshold is None:
        threshold = CE_LONG_DEGREE
    if threshold <= 0:
        return torch.arange(deg.numel(), device=deg.device), 0
    longr = deg > threshold
    order = torch.cat([torch.nonzero(longr).flatten(), torch.nonzero(~longr).flatten()])
    return order, int(longr.sum())


def spmm_ce(rowptr, col, Z, C, rscale, bias, labels, mask, inv_count, mode=0, G=None, init=None, gslot=None,
            db_out=None, n_long=0, stats_out=None, bump=None):
    """Layer-2 aggregate + log-softmax + NLL.  Returns (stats[68] summed, G).
    ``init`` (optional fp32 [n, >=C]): partial sums of other edges.
    ``gslot`` (optional int32 [n]): G is compact -- row i (a train row, gslot[i] >= 0)
    goes to G[gslot[i]], other rows (whose dlogits are zero) are not written.
    ``db_out`` (optional fp32 [C], GPU): the per-class dlogits sums (the bias gradient,
    stats[4:4 + C]) are also summed straight into it -- a second fixed-order pass over
    the partials instead of a device-to-device copy.
    ``n_long``: rows [0, n_long) are long rows the caller ordered first; the GPU kernel
    gives each of them a whole wave (see ``long_row_order``).  Results do not depend on it.
    ``stats_out`` = (buffer, index) (GPU): ONE fixed-order reduction writes column c of
    the 68 to buffer[index[c]] (index < 0: dropped) and that buffer is returned -- e.g.
    the loss / accuracy sums to a scratch tail and the per-class dlogits sums straight
    into the bias gradient, with no copy or second pass."""
    if checks.enabled():
        checks.csr(rowptr, col, Z.shape[0], "spmm_ce")
        checks.rows(labels, rowptr.numel() - 1, "spmm_ce labels")
        checks.rows(mask, rowptr.numel() - 1, "spmm_ce mask")
    n = rowptr.numel() - 1
    ld = Z.shape[1]
    if Z.is_cuda:
        hip = native.hip()
        nb = hip.gnn_spmm_ce_blocks(n, int(n_long))
        stats = torch.empty(nb, 68, dtype=torch.float32, device=Z.device)
        if G is None and mode == 0:
            if gslot is not None:
                raise ValueError("a compact G (gslot) must be allocated by the caller")
            G = torch.empty(n, ld, dtype=torch.bfloat16, device=Z.device)
        if gslot is not None and gslot.dtype != torch.int32:
            raise TypeError("gslot must be int32")
        hip.gnn_spmm_ce(rowptr.data_ptr(), col.data_ptr(), Z.data_ptr(), rscale.data_ptr(), bias.data_ptr(),
                        labels.data_ptr(), mask.data_ptr(), stats.data_ptr(), G.data_ptr() if G is not None else 0,
                        init.data_ptr() if init is not None else 0, init.shape[1] if init is not None else 0,
                        n, C, ld, mode, float(inv_count), _st(Z),
                        gslot.data_ptr() if gslot is not None else 0, int(n_long))
        if stats_out is not None:
            buf, index = stats_out
            slab_sum(stats, buf, index=index)
            return buf, G
        out = torch.empty(68, dtype=torch.float32, device=Z.device)
        slab_sum(stats, out)
        if db_out is not None:
            key = (Z.device, C)
            idx = _DB_INDEX.get(key)
            if idx is None:
                c = torch.arange(68, dtype=torch.int32)
                idx = _DB_INDEX[key] = torch.where((c >= 4) & (c < 4 + C), c - 4, -1).to(torch.int32).to(Z.device)
            slab_sum(stats, db_out, index=idx, bump=bump)
        elif bump is not None:
            raise ValueError("spmm_ce: bump rides on the db_out reduction")
        return out, G
    rows = _row_ids(rowptr)
    acc = torch.zeros(n, C, dtype=torch.float32)
    acc.index_add_(0, rows, Z[col.long(), :C].float())
    if init is not None:
        acc = acc + init[:n, :C].float()
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
        gval = (dl * rscale[:, None]).to(Z.dtype)
        if gslot is not None:
            sel = gslot >= 0
            G[gslot[sel].long(), :C] = gval[sel].to(G.dtype)
            G[gslot[sel].long(), C:] = 0
        else:
            if G is None:
                G = torch.zeros(n, ld, dtype=Z.dtype)
            G.zero_()
            G[:, :C] = gval.to(G.dtype)
    return stats, G


_STAGE = {}


def slab_sum(P, out, index=None, groups=None, bump=None):
    """out[index[c]] = sum_r P[r, c] (``index`` None: out[c]; index < 0: dropped) -- the
    fixed-order column sum of per-block partials (deterministic, no atomics), in one pass
    or, for more than 256 rows, two (``groups`` row groups: 512 above 4096 rows, else one
    group per 32 rows -- a one-pass sum of a few thousand rows is a serial load chain per
    lane in the two blocks of a 68-column reduce, 14 us on arxiv's cross-entropy stats).
    On the CPU: the same sums with torch.
    ``bump`` (GPU, int32[1]): incremented by the final pass (a step counter advanced
    without a launch of its own)."""
    S, W = P.shape
    if not P.is_cuda:
        v = P.sum(0)
        if index is None:
            out[:W] = v
        else:
            keep = index >= 0
            out[index[keep].long()] = v[keep]
        return out
    if not (P.dtype == torch.float32 and out.dtype == torch.float32 and P.is_contiguous()):
        raise TypeError("slab_sum: contiguous fp32 partials and fp32 output expected")
    if index is not None and (index.dtype != torch.int32 or index.numel() != W):
        raise TypeError("slab_sum: index must be int32 of the partials' width")
    G = groups if groups is not None else (512 if S > 4096 else (-(-S // 32) if S > 256 else 1))
    stage = None
    if G > 1:
        key = (P.device, G * W)
        stage = _STAGE.get(key)
        if stage is None:
            stage = _STAGE[key] = torch.empty(G * W, dtype=torch.float32, device=P.device)
    native.hip().gnn_slab_sum(P.data_ptr(), S, W, stage.data_ptr() if stage is not None else 0, G,
                              out.data_ptr(), index.data_ptr() if index is not None else 0, _st(P),
                              bump.data_ptr() if bump is not None else 0)
    return out


def tall_gemm_tn(A: torch.Tensor, B: torch.Tensor, chunk: int = 8192) -> torch.Tensor:
    """A^T B (fp32) for tall A [M, k1], B [M, k2] with tiny k1 x k2: a plain GEMM
    would give the whole M-long reduction to k1*k2/tile^2 workgroups (16 for
    256 x 256 on 64 x 64 tiles -- 6 % of the CUs); instead split K into row
    chunks as ONE batched GEMM with fp32 partials and sum them in fixed order."""
    M = A.shape[0]
    S = M // chunk
    cuda = A.is_cuda
    out = None
    if S:
        a = A[:S * chunk].reshape(S, chunk, A.shape[1]).transpose(1, 2)
        b = B[:S * chunk].reshape(S, chunk, B.shape[1])
        if cuda and A.dtype != torch.float32:
            out = torch.bmm(a, b, out_dtype=torch.float32).sum(0)
        else:
            out = torch.bmm(a.float(), b.float()).sum(0)
    if M > S * chunk:
        a, b = A[S * chunk:], B[S * chunk:]
        if cuda and A.dtype != torch.float32:
            tail = torch.mm(a.t(), b, out_dtype=torch.float32)
        else:
            tail = a.float().t() @ b.float()
        out = tail if out is None else out + tail
    return out


DROP_BIT_CTR = 0x80000000


def dropout_keep_mask(rows: int, F: int, p: float, key, step, row0: int = 0) -> torch.Tensor:
    """Keep mask of the fused dropout (host mirror of cgnn_common.h drop_draw /
    drop_keep16).  Element (row, n), n = 32 t + 8 g + 4 h + i, q = 4 g + i:
      byte mode (any p): byte q of the Philox draw keyed (row, 2 t + h, step), kept if
      >= thr8 = round(256 p);
      bit mode (p = 1/2, thr8 = 128): bit 16 (t % 8) + q of the draw keyed
      (row, DROP_BIT_CTR + 2 (t // 8) + h, step), kept if set (one bit per decision)."""
    import numpy as np
    thr8 = min(255, int(np.floor(p * 256.0 + 0.5)))
    if thr8 == 0:
        return torch.ones(rows, F, dtype=torch.bool)
    r = (row0 + np.arange(rows)).astype(np.uint32)[:, None]
    n = np.arange(F)
    t, h = n // 32, (n // 4) % 2
    q = (n % 4) + 4 * ((n % 32) // 8)
    if thr8 == 128:
        ctr = (DROP_BIT_CTR + 2 * (t // 8) + h).astype(np.uint32)[None, :]
        b = 16 * (t % 8) + q
    else:
        ctr = (2 * t + h).astype(np.uint32)[None, :]
        b = 8 * q
    words = np.stack(philox.philox4x32_10(r, ctr, step, philox.RNG_DROPOUT, key[0], key[1]), -1)
    wsel = np.take_along_axis(words, (b // 32)[None, :, None].repeat(rows, 0), -1)[..., 0]
    bits = wsel >> (b % 32).astype(np.uint32)[None, :]
    if thr8 == 128:
        return torch.from_numpy((bits & 1) == 1)
    return torch.from_numpy((bits & 0xFF) >= thr8)


def bias_relu_dropout_(H, bias, F, p, key, step, row0=0):
    """In place: H = dropout(relu(H + bias)); the mask is keyed by the GLOBAL row
    (row0 + local row), so it does not depend on how rows are partitioned."""
    if H.is_cuda:
        native.hip().gnn_bias_relu_dropout(H.data_ptr(), bias.data_ptr(), H.shape[0], F, H.shape[1],
                                           float(p), int(key[0]), int(key[1]), int(step), int(row0), _st(H))
        return H
    x = torch.relu(H[:, :F].float() + bias[:F])
    if p > 0:
        keep = dropout_keep_mask(H.shape[0], F, p, key, step, row0)
        x = torch.where(keep, x / (1 - p), torch.zeros_like(x))
    H.zero_()
    H[:, :F] = x.to(H.dtype)
    return H


def _step_args(step):
    """(scalar step, device pointer): a device int32 tensor is read by the kernel at
    launch time (hipGraph replays see the current value), an int is passed by value."""
    if isinstance(step, torch.Tensor):
        return 0, step.data_ptr()
    return int(step), 0


def _step_value(step):
    return int(step.item()) if isinstance(step, torch.Tensor) else int(step)


def keep_image(n, hidden, device):
    """Buffer of a keep image (the dropout masks of an n-row, ``hidden``-wide GCN layer as
    the fused backward reads them: 1 bit per element, whole 32-row tiles)."""
    hw = native.hip().gnn_keep_image_halfwords(int(n), int(hidden))
    return torch.empty(hw, dtype=torch.int16, device=device)


def draw_keep_image(kimg, n, hidden, p, key, step, row0=0):
    """Fill ``kimg`` with the masks dense_fwd draws for the same (n, p, key, step, row0)."""
    sv, sp = _step_args(step)
    rc = native.hip().gnn_keep_image(kimg.data_ptr(), int(n), int(hidden), float(p), int(key[0]), int(key[1]), sv,
                                     int(row0), _st(kimg), step_ptr=sp)
    if rc != 0:
        raise RuntimeError("gnn_keep_image failed (%d)" % rc)
    return kimg


def dense_fwd(AX, W1, b1, W2, dinv, H1, Z2, F, p, key, step, row0=0, kimg=None):
    """H1 = dropout(relu(AX[:, :F] W1 + b1)), Z2 = dinv * (H1 W2) (fused MFMA kernel on GPU).
    ``H1=None`` (GPU only): H1 is not stored -- the fused backward recomputes it.
    ``step``: the dropout step, an int or a device int32[1] tensor.  ``kimg`` (GPU, a
    ``keep_image`` buffer): also write the dropout masks for the fused backward."""
    n = Z2.shape[0]
    HD, C = W1.shape[1], W2.shape[1]
    if AX.is_cuda:
        sv, sp = _step_args(step)
        rc = native.hip().gnn_dense_fwd(AX.data_ptr(), W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                                        dinv.data_ptr(), H1.data_ptr() if H1 is not None else 0,
                                        Z2.data_ptr(), n, F, AX.shape[1],
                                        HD, C, Z2.shape[1], float(p), int(key[0]), int(key[1]), sv,
                                        int(row0), _st(AX), step_ptr=sp,
                                        kimg=kimg.data_ptr() if kimg is not None else 0)
        if rc == 0:
            return True
        if rc != -1:
            raise RuntimeError("gnn_dense_fwd failed (%d)" % rc)
        return False          # shape not covered by a compiled variant
    H1.copy_((AX[:n, :F].float() @ W1.to(torch.bfloat16).float()).to(torch.bfloat16))
    bias_relu_dropout_(H1, b1, HD, p, key, _step_value(step), row0)
    y2 = H1.float() @ W2.to(torch.bfloat16).float()
    Z2.zero_()
    Z2[:, :C] = (y2 * dinv[:n, None]).to(torch.bfloat16)
    return True


def dense_bwd(dY2, W2, H1, dP1, p):
    """dP1 = (dY2 W2^T) * [H1 > 0] / (1-p)."""
    n = dP1.shape[0]
    HD, C = W2.shape
    if dY2.is_cuda:
        rc = native.hip().gnn_dense_bwd(dY2.data_ptr(), W2.data_ptr(), H1.data_ptr(), dP1.data_ptr(), n,
                                        HD, C, dY2.shape[1], float(p), _st(dY2))
        if rc == 0:
            return True
        if rc != -1:
            raise RuntimeError("gnn_dense_bwd failed (%d)" % rc)
        return False
    g = dY2[:n, :C].float() @ W2.to(torch.bfloat16).float().t()
    dP1.copy_(torch.where(H1[:n].float() > 0, g / (1 - p), torch.zeros_like(g)).to(torch.bfloat16))
    return True


def fused_bwd_supported(F, hidden, C):
    """Whether a compiled fused-backward variant covers F features (+ the ones column),
    ``hidden`` units and C classes (the row pitches only need to cover them)."""
    return bool(native.hip().gnn_fused_bwd_supported(int(F) + 1, int(hidden), int(C)))


def fused_bwd(AX, dY2, W1, b1, W2, n, F, p, key, step, row0=0, gpart=None, grads=None, grad_index=None,
              kimg=None):
    """Fused GCN dense backward (GPU): recomputes H1 from AX, then
    dP1 = (dY2 W2^T) * [H1 > 0] / (1-p) and the weight gradients in one pass.
    The dropout masks come from ``kimg``, the keep image the forward wrote
    (``dense_fwd(..., kimg=)``); without one they are drawn here from (key, step, row0).
    Returns (gW1 [F, HD], gb1 [HD], gW2 [HD, C], gpart); with ``grads`` (the flat fp32
    gradient buffer, gW1 | gb1 | gW2 at its start) the sums are written there instead
    and (None, None, None, gpart) is returned."""
    hip = native.hip()
    HD, C = W1.shape[1], W2.shape[1]
    ldx = AX.shape[1]
    nb, width = hip.gnn_fused_bwd_blocks(n), hip.gnn_fused_bwd_width(F + 1)
    if gpart is None or gpart.shape != (nb, HD, width):
        gpart = torch.empty(nb, HD, width, dtype=torch.float32, device=AX.device)
    if p > 0 and kimg is None:
        kimg = draw_keep_image(keep_image(n, HD, AX.device), n, HD, p, key, step, row0)
    rc = hip.gnn_fused_bwd(AX.data_ptr(), dY2.data_ptr(), W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                           kimg.data_ptr() if kimg is not None else 0, gpart.data_ptr(), n, F, ldx, HD, C,
                           dY2.shape[1], float(p), _st(AX))
    if rc != 0:
        raise RuntimeError("gnn_fused_bwd failed (%d)" % rc)
    if grads is not None:
        # fixed-order reduction over the block slabs, scattered straight into the flat
        # gradient buffer [gW1 (F x HD) | gb1 | gW2 (HD x C) | ...]
        if grad_index is None:
            grad_index = fused_bwd_grad_index(F, HD, C, width, device=AX.device)
        slab_sum(gpart.view(nb, HD * width), grads, grad_index)
        return None, None, None, gpart
    g = gpart.sum(0)                     # fixed-order reduction over the block slabs
    kf = width - 64
    return g[:, :F].t(), g[:, F], g[:, kf:kf + C], gpart


def fused_bwd_width(F):
    """Row width of a fused-backward slab for F features (+ the ones column)."""
    return native.hip().gnn_fused_bwd_width(int(F) + 1)


def fused_bwd_grad_index(F, HD, C, width, device=None):
    """Destination in the flat gradient buffer [gW1 (F x HD) | gb1 (HD) | gW2 (HD x C)] of
    every element (h, j) of a fused-backward slab [HD][width] (-1: padding)."""
    kf = width - 64
    h = torch.arange(HD).view(HD, 1)
    j = torch.arange(width).view(1, width)
    n1 = F * HD
    idx = torch.full((HD, width), -1, dtype=torch.int64)
    idx = torch.where(j < F, j * HD + h, idx)
    idx = torch.where(j == F, n1 + h, idx)
    idx = torch.where((j >= kf) & (j < kf + C), n1 + HD + h * C + (j - kf), idx)
    return idx.view(-1).to(torch.int32).to(device)


def relu_dropout_bwd_(dH, H, p):
    if dH.is_cuda:
        native.hip().gnn_relu_dropout_bwd(dH.data_ptr(), H.data_ptr(), dH.numel(), float(p), _st(dH))
        return dH
    dH.copy_(torch.where(H.float() > 0, dH.float() / (1 - p), torch.zeros_like(dH, dtype=torch.float32)).to(dH.dtype))
    return dH


_ADAM_DONE = {}


def adam_(param, grad, m, v, lr, step_t, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, step_done=False):
    """PyTorch-semantics Adam on flat fp32 buffers; ``step_t`` is a device int32[1]
    holding the number of completed steps (incremented here).  On a GPU, for up to 256
    blocks of parameters, the kernel's last-arriving block increments it (a zeroed
    arrival counter kept per step tensor) instead of a separate launch: the GCN epoch
    +0.3 % (profiles/r06_sage/adam_fold).  Larger grids keep the launch -- 1.2 K blocks
    counting on one address measured slower (GraphSAGE).  ``step_done`` (GPU): a
    reduction before this update already advanced ``step_t`` (slab_sum's bump)."""
    if param.is_cuda and step_done:
        native.hip().gnn_adam(param.data_ptr(), m.data_ptr(), v.data_ptr(), grad.data_ptr(), param.numel(),
                              float(lr), float(b1), float(b2), float(eps), float(wd), step_t.data_ptr(),
                              _st(param), 0, 1)
        return param
    if param.is_cuda:
        fold = param.numel() <= 256 * 256
        done = None
        if fold:
            key = (step_t.device.index, step_t.data_ptr())
            done = _ADAM_DONE.get(key)
            if done is None:
                done = _ADAM_DONE[key] = torch.zeros(1, dtype=torch.int32, device=step_t.device)
        native.hip().gnn_adam(param.data_ptr(), m.data_ptr(), v.data_ptr(), grad.data_ptr(), param.numel(),
                              float(lr), float(b1), float(b2), float(eps), float(wd), step_t.data_ptr(),
                              _st(param), done.data_ptr() if fold else 0)
        if not fold:
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
