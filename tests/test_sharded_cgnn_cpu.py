"""Long-N CGNN: one job's samples split over gloo ranks (engine/sharded.py) equals
the single-process run -- noise keyed by the global sample, MMD rows vs all
columns, SUM-all-reduced parameter gradients, all-reduced loss."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cgnn_amd.engine.program import program_for_dag, program_for_pair
from cgnn_amd.engine.reference import ReferenceTrainer
from cgnn_amd.engine.sharded import SampleShardedTrainer, shard_range
from cgnn_amd.utils.graph import DirectedGraph
from cgnn_amd.utils.philox import model_key


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _job(N, kind):
    rng = np.random.default_rng(0)
    if kind == "pair":
        x = rng.standard_normal(N)
        y = np.tanh(x) + 0.3 * rng.standard_normal(N)
        return program_for_pair(8), np.stack([x, y]).astype(np.float32)
    g = DirectedGraph()
    for a, b in [("A", "B"), ("B", "C")]:
        g.add(a, b)
    a = rng.standard_normal(N)
    b = a ** 2 + 0.3 * rng.standard_normal(N)
    c = np.sin(b) + 0.3 * rng.standard_normal(N)
    return program_for_dag(g, 8), np.stack([a, b, c]).astype(np.float32)


def _worker(rank, world, port, N, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prog, data = _job(N, kind)
    r0, n = shard_range(N, rank, world)
    tr = SampleShardedTrainer([prog], [data[:, r0:r0 + n]], [model_key(3, kind)], 8, "cpu", N)
    out[rank] = tr.run(*_steps(N))
    dist.destroy_process_group()


def _steps(N):
    return (1, 1) if N > 5000 else (2, 1)


@pytest.mark.parametrize("N,world,kind", [(20000, 2, "pair"), (600, 3, "dag")])
def test_sample_sharded_cgnn_matches_single_process(N, world, kind):
    prog, data = _job(N, kind)
    single = SampleShardedTrainer([prog], [data], [model_key(3, kind)], 8, "cpu", N).run(*_steps(N))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), N, kind, out), nprocs=world, join=True)
    for r in range(world):
        np.testing.assert_allclose(out[r], single, rtol=1e-9)
    if N <= 1000:      # and the unsharded oracle trainer (exact dense MMD) agrees
        ref = ReferenceTrainer([prog], [data], [model_key(3, kind)], 8).run(2, 1)
        np.testing.assert_allclose(single, ref, rtol=1e-9)
