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


def selftest(device, group=None, rows: int = 1 << 12, width: int = 64) -> dict:
    """Content-checked round of the collectives the trainers use -- all_to_all_single
    with uneven splits, all_gather_into_tensor, async all_reduce waited on a side
    stream, broadcast -- before a timed run.  Every rank fills its buffers with
    values that encode (rank, position), so a mis-wired launch (wrong world size,
    ranks on one device, a transport that drops or reorders) fails loudly here
    instead of producing a number.  Raises RuntimeError on a mismatch; returns
    {"backend", "world_size", "ms"}."""
    import time
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gloo = dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if gloo else torch.device(device)      # gloo: host tensors
    f32 = dict(dtype=torch.float32, device=dev)
    i64 = dict(dtype=torch.int64, device=dev)
    t0 = time.perf_counter()

    def enc(src, dst, n):        # value of row k of the slice src sends to dst
        return (src * 4096 + dst) * (1 << 20) + torch.arange(n, **i64)

    # all_to_all_single, rank r sends (r + p + 1) rows to peer p
    send_sizes = [rank + p + 1 for p in range(world)]
    recv_sizes = [p + rank + 1 for p in range(world)]
    send = torch.cat([enc(rank, p, send_sizes[p]) for p in range(world)])[:, None].repeat(1, width).contiguous()
    recv = torch.empty(sum(recv_sizes), width, **i64)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_sizes, input_split_sizes=send_sizes, group=group)
    want = torch.cat([enc(p, rank, recv_sizes[p]) for p in range(world)])[:, None].expand(-1, width)
    bad = [("all_to_all_single", recv, want)]
    # all_gather_into_tensor (gloo: the list form)
    loc = enc(rank, 0, rows)
    if gloo:
        parts = [torch.empty(rows, **i64) for _ in range(world)]
        dist.all_gather(parts, loc, group=group)
        gat = torch.cat(parts)
    else:
        gat = torch.empty(world * rows, **i64)
        dist.all_gather_into_tensor(gat, loc, group=group)
    want_g = torch.cat([enc(p, 0, rows) for p in range(world)])
    bad.append(("all_gather_into_tensor", gat, want_g))
    # async all_reduce, consumed on a side stream after wait() (the trainers' overlap pattern)
    red = torch.full((rows, width), float(rank + 1), **f32)
    work = dist.all_reduce(red, group=group, async_op=True)
    if dev.type == "cuda":
        side = torch.cuda.Stream(dev)
        with torch.cuda.stream(side):
            work.wait()
            red2 = red * 2
        torch.cuda.current_stream(dev).wait_stream(side)
    else:
        work.wait()
        red2 = red * 2
    bad.append(("all_reduce(async)", red2, torch.full((rows, width), float(world * (world + 1)), **f32)))
    # broadcast from the last rank
    b = torch.full((rows,), float(rank), **f32)
    dist.broadcast(b, world - 1, group=group)
    bad.append(("broadcast", b, torch.full((rows,), float(world - 1), **f32)))
    for name, got, want in bad:
        if not torch.equal(got, want):
            raise RuntimeError("collective self-test: %s returned wrong data on rank %d of %d (backend %s)"
                               % (name, rank, world, dist.get_backend(group)))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return {"backend": dist.get_backend(group), "world_size": world,
            "ms": round(1e3 * (time.perf_counter() - t0), 2)}
