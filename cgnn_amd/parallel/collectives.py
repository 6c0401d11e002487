"""Differentiable row collectives for graph-sharded models (one process per GPU,
RCCL over xGMI; gloo on CPUs).

A graph whose rows are partitioned in contiguous blocks of ``per`` rows needs
the source-side activations of every rank: ``gather_rows`` all-gathers them in
the forward and reduce-scatters their gradients back to the owners in the
backward (every rank's edges contribute to remote rows).  One ring collective
per direction and layer -- bandwidth-optimal on xGMI's point-to-point links,
and with random-ish partitions the halo of a rank is most of the graph anyway.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _pad_rows(x: torch.Tensor, rows: int) -> torch.Tensor:
    if x.shape[0] == rows:
        return x.contiguous()
    out = torch.zeros((rows,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    out[:x.shape[0]] = x
    return out


def all_gather_rows(x_local: torch.Tensor, per: int, n_global: int, group=None) -> torch.Tensor:
    world = dist.get_world_size(group)
    out = torch.empty((per * world,) + tuple(x_local.shape[1:]), dtype=x_local.dtype, device=x_local.device)
    dist.all_gather_into_tensor(out, _pad_rows(x_local, per), group=group)
    return out[:n_global]


def reduce_scatter_rows(x_full: torch.Tensor, per: int, n_local: int, group=None) -> torch.Tensor:
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    full = _pad_rows(x_full, per * world)
    if dist.get_backend(group) == "gloo":            # gloo has no reduce-scatter
        dist.all_reduce(full, group=group)
        return full[rank * per: rank * per + n_local].clone()
    out = torch.empty((per,) + tuple(x_full.shape[1:]), dtype=x_full.dtype, device=x_full.device)
    dist.reduce_scatter_tensor(out, full, group=group)
    return out[:n_local]


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_local, per, n_global, group):
        ctx.per, ctx.n_local, ctx.group = per, x_local.shape[0], group
        return all_gather_rows(x_local, per, n_global, group)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_rows(g.contiguous(), ctx.per, ctx.n_local, ctx.group), None, None, None


def gather_rows(x_local: torch.Tensor, per: int, n_global: int, group=None) -> torch.Tensor:
    """Rows of all ranks ([n_global, ...]) from this rank's block; the backward
    sums every rank's gradient of a row into its owner."""
    return _GatherRows.apply(x_local, per, n_global, group)
