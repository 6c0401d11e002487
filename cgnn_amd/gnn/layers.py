"""Autograd building blocks for GNNs of any depth on the HIP kernels -- GNN
track, not in the reference.

* ``norm_aggregate`` -- ``Y = D^-1/2 (A+I) D^-1/2 X`` on the CSR of A + I.  The
  column scale is applied in the gather (one float per gathered row), the row
  scale in the SpMM epilogue, so no per-edge value is read.  The normalised adjacency is
  symmetric, so the backward is the same SpMM on the incoming gradient (no
  transposed CSR).
* ``gcn_layer`` / ``GCNConv`` -- ``act(Â (H W) + b)`` (transform first: the
  gathered rows are the narrower of the two widths) with the normalisation,
  bias and ReLU inside the SpMM and a split-K weight gradient.
* ``GCN`` -- L layers with ReLU + dropout between them.

Everything runs on the same ``ops.spmm`` as the fused 2-layer trainer (HIP on
GPU tensors, PyTorch index ops on CPU tensors); dense products are hipBLASLt
GEMMs.  Storage dtype follows the input (fp32 / bf16 / fp16); aggregation
accumulates in fp32.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from . import ops


def pad_cols(x: torch.Tensor, mult: int = 8) -> torch.Tensor:
    F = x.shape[1]
    return x if F % mult == 0 else torch.nn.functional.pad(x, (0, mult - F % mult))


class NormGraph:
    """CSR of A + I with the symmetric normalisation vector ``dinv``."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, dinv: torch.Tensor):
        self.rowptr, self.col, self.dinv = rowptr.contiguous(), col.contiguous(), dinv.contiguous()
        self.n = rowptr.numel() - 1

    @classmethod
    def from_data(cls, g) -> "NormGraph":
        return cls(g.rowptr, g.col, g.dinv)


def aggregate(x: torch.Tensor, g: NormGraph, prescaled: bool = False, bias=None, relu: bool = False):
    """act(dinv * (A+I) (dinv * x) + bias) in the storage dtype of x; ``prescaled``:
    x already carries the column scale.  Bias / ReLU run in the SpMM epilogue."""
    F = x.shape[1]
    xs = pad_cols(x).contiguous()
    out = ops.spmm(g.rowptr, g.col, xs, F, rscale=g.dinv, bias=bias, relu=relu, out_dtype=x.dtype,
                   ld_out=xs.shape[1], cscale=None if prescaled else g.dinv)
    return out[:, :F] if out.shape[1] != F else out


class _NormAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g: NormGraph):
        ctx.g = g
        return aggregate(x, g)

    @staticmethod
    def backward(ctx, gy):
        return aggregate(gy.contiguous(), ctx.g), None


def norm_aggregate(x: torch.Tensor, g: NormGraph) -> torch.Tensor:
    return _NormAggregate.apply(x, g)


class _GCNLayer(torch.autograd.Function):
    """``act(Â (H W) + b)`` with the normalisation, bias and ReLU inside the SpMM
    (column scale in the gather, row scale + bias + ReLU in the epilogue).
    Backward: ReLU mask, ``db = sum dY``, ``dZ = Â dY`` (same SpMM, Â symmetric),
    ``dW = H^T dZ`` as a split-K batched GEMM (``ops.tall_gemm_tn``), ``dH = dZ W^T``."""

    @staticmethod
    def forward(ctx, h, W, b, g: NormGraph, relu: bool):
        Wc = W.to(h.dtype)
        z = h @ Wc
        out_dim = z.shape[1]
        zp = pad_cols(z).contiguous()
        y = ops.spmm(g.rowptr, g.col, zp, out_dim, rscale=g.dinv, cscale=g.dinv, bias=b.float().contiguous(),
                     relu=relu, out_dtype=h.dtype, ld_out=zp.shape[1])
        if y.shape[1] != out_dim:
            y = y[:, :out_dim]
        ctx.g, ctx.relu = g, relu
        ctx.save_for_backward(h, Wc, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, Wc, y = ctx.saved_tensors
        g = ctx.g
        dy = dy.contiguous()
        if ctx.relu:
            dy = torch.ops.aten.threshold_backward(dy, y, 0)
        db = dy.float().sum(0)
        out_dim = dy.shape[1]
        dyp = pad_cols(dy).contiguous()
        dz = ops.spmm(g.rowptr, g.col, dyp, out_dim, rscale=g.dinv, cscale=g.dinv, out_dtype=dy.dtype,
                      ld_out=dyp.shape[1])
        if dz.shape[1] != out_dim:
            dz = dz[:, :out_dim]
        dW = ops.tall_gemm_tn(h, dz)
        dh = dz @ Wc.t() if ctx.needs_input_grad[0] else None
        return dh, dW, db, None, None


def gcn_layer(h: torch.Tensor, W: torch.Tensor, b: torch.Tensor, g: NormGraph, relu: bool) -> torch.Tensor:
    return _GCNLayer.apply(h, W, b, g, relu)


class GCNConv(torch.nn.Module):
    """``Â (H W) + b``; glorot-uniform W, zero b (the PyG GCNConv initialisation)."""

    def __init__(self, in_dim: int, out_dim: int, generator: Optional[torch.Generator] = None):
        super().__init__()
        bound = math.sqrt(6.0 / (in_dim + out_dim))
        self.weight = torch.nn.Parameter((torch.rand(in_dim, out_dim, generator=generator) * 2 - 1) * bound)
        self.bias = torch.nn.Parameter(torch.zeros(out_dim))

    def forward(self, h: torch.Tensor, g: NormGraph, relu: bool = False) -> torch.Tensor:
        return gcn_layer(h, self.weight, self.bias, g, relu)


class GCN(torch.nn.Module):
    """L-layer GCN: ``dims = [in, hidden..., out]``; ReLU + dropout between layers."""

    def __init__(self, dims: Sequence[int], dropout: float = 0.5, seed: int = 0):
        super().__init__()
        gen = torch.Generator().manual_seed(seed)
        self.dims = list(dims)
        self.convs = torch.nn.ModuleList(GCNConv(a, b, gen) for a, b in zip(dims[:-1], dims[1:]))
        self.dropout = float(dropout)

    def forward(self, x: torch.Tensor, g: NormGraph) -> torch.Tensor:
        h = x
        L = len(self.convs)
        for k, conv in enumerate(self.convs):
            h = conv(h, g, relu=k < L - 1)
            if k < L - 1 and self.training and self.dropout > 0:
                h = torch.nn.functional.dropout(h, self.dropout)
        return h
