"""Operand validation before hand-written kernel launches (``CGNN_CHECK=1``).

The gather kernels trust their index operands: a CSR column, a gather-on-load row
index or a halo row index outside its matrix is an out-of-bounds device access (on
this hardware a fault can take the GPU down for every job on the node, and GPU
sanitizers are not available).  With ``CGNN_CHECK=1`` every op validates, on the
device, before launching: CSR ``rowptr`` starts at 0, never decreases and stays
within ``col``; every used column index lies in ``[0, n_src)``; row indices lie in
their matrix; operand row counts cover what the grid reads.  A violation raises a
``ValueError`` naming the op.  Off by default (each check synchronises to read one
reduction); the CPU suite and a GPU test run whole training steps with it on.
"""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get("CGNN_CHECK", "0") not in ("", "0")


def enabled() -> bool:
    return ENABLED


def _fail(what, msg):
    raise ValueError("CGNN_CHECK: %s: %s" % (what, msg))


def csr(rowptr: torch.Tensor, col: torch.Tensor, n_src: int, what: str, n_rows: int = None):
    """rowptr[0] == 0, non-decreasing, rowptr[-1] <= len(col); col[:nnz] in [0, n_src)."""
    if not ENABLED:
        return
    if rowptr.dim() != 1 or rowptr.numel() < 1:
        _fail(what, "rowptr must be a non-empty vector")
    if n_rows is not None and rowptr.numel() - 1 != n_rows:
        _fail(what, "rowptr describes %d rows, expected %d" % (rowptr.numel() - 1, n_rows))
    rp = rowptr.long()
    if int(rp[0]) != 0:
        _fail(what, "rowptr[0] = %d" % int(rp[0]))
    if rp.numel() > 1 and bool((rp[1:] < rp[:-1]).any()):
        _fail(what, "rowptr decreases")
    nnz = int(rp[-1])
    if nnz > col.numel():
        _fail(what, "rowptr ends at %d but col has %d entries" % (nnz, col.numel()))
    if nnz:
        c = col[:nnz]
        lo, hi = int(c.min()), int(c.max())
        if lo < 0 or hi >= n_src:
            _fail(what, "column index range [%d, %d] outside [0, %d)" % (lo, hi, n_src))


def index(idx: torch.Tensor, n: int, what: str):
    """Every entry of ``idx`` in [0, n)."""
    if not ENABLED or idx is None or idx.numel() == 0:
        return
    lo, hi = int(idx.min()), int(idx.max())
    if lo < 0 or hi >= n:
        _fail(what, "index range [%d, %d] outside [0, %d)" % (lo, hi, n))


def rows(t: torch.Tensor, n: int, what: str):
    """``t`` has at least ``n`` rows."""
    if ENABLED and t is not None and t.shape[0] < n:
        _fail(what, "operand has %d rows, the launch reads %d" % (t.shape[0], n))
