"""The multi-rank GCN code paths through RCCL itself (the driver's 8-GPU scaling run
is the first multi-GPU launch; every earlier multi-rank test used gloo).  One
process, a 1-rank ``nccl`` group, and ``GCNTrainer(collectives=True)`` forcing the
exchange branches: the async all-gather / all-to-all on RCCL's stream, the wait before
the remote edges, the split aggregation through the fp32 partial, the backward
all-gather overlap and the gradient all-reduce.  With one rank every exchange is the
identity, so the run must reproduce the plain one-GPU trainer."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def nccl_group():
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        yield dist
    finally:
        dist.destroy_process_group()
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)


def test_collective_selftest_on_rccl(nccl_group):
    from cgnn_amd.parallel.collectives import selftest
    res = selftest("cuda:0")
    assert res["backend"] == "nccl" and res["world_size"] == 1


@pytest.mark.parametrize("halo", [False, True])
def test_gcn_multirank_branches_through_rccl(nccl_group, halo):
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    g = synthetic("ogbn-products", seed=2, device="cuda:0", scale=0.003)
    ref = GCNTrainer(g, hidden=256, rank=0, world=1)
    forced = GCNTrainer(g, hidden=256, rank=0, world=1, collectives=True, halo=halo)
    assert not ref.multi and forced.multi and forced.halo == halo
    assert forced.AX_next is not None and forced._bwd_overlap
    for _ in range(4):
        ref.train_step()
        forced.train_step()
    lr, lf = ref.train_loss(), forced.train_loss()
    # training takes the one-pass layer-2 and backward aggregations after the exchanges
    # (round 6) and the layer-1 SpMM in two row halves: the same sums in the same order as
    # the one-GPU path, so the whole update is bitwise equal
    assert lr == lf, (lr, lf)
    assert torch.equal(forced.params, ref.params)
    a, b = ref.evaluate(), forced.evaluate()
    assert abs(a["val_acc"] - b["val_acc"]) < 5e-3
