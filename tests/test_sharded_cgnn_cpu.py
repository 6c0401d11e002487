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


def _pair_data(N):
    rng = np.random.default_rng(1)
    a = rng.standard_normal(N)
    b = np.tanh(a) + 0.3 * rng.standard_normal(N)
    return a, b


_KW = dict(nb_runs=1, train_epochs=1, test_epochs=1, max_nb_points=None, gpu=False, h_layer_dim=8)


def _api_worker(rank, world, port, N, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cgnn
    a, b = _pair_data(N)
    out[rank] = cgnn.GNN().predict_proba(a, b, **_KW)
    dist.destroy_process_group()


def test_public_api_long_n_pairwise_sample_sharded(monkeypatch):
    """``GNN().predict_proba`` with subsampling off (max_nb_points=None) and N (6000) above
    ``long_n_min``: the jobs go to the sample-sharded trainer; 2 gloo ranks (each owning
    half the samples of every job) give the one-process score."""
    import cgnn
    from cgnn_amd.engine import scorer
    N = 6000
    calls = []
    real = scorer._run_long

    def spy(jobs, cfg):
        calls.append((len(jobs), jobs[0].data.shape))
        return real(jobs, cfg)
    monkeypatch.setattr(scorer, "_run_long", spy)
    a, b = _pair_data(N)
    single = cgnn.GNN().predict_proba(a, b, **_KW)
    assert calls == [(2, (2, N))], calls             # the run's A->B and B->A models, all samples
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_api_worker, args=(2, _free_port(), N, out), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_allclose(out[r], single, rtol=1e-9)
    # the reference's cap (1500) keeps the batched engine
    calls.clear()
    cgnn.GNN().predict_proba(a[:3000], b[:3000], **dict(_KW, max_nb_points=1500))
    assert calls == []
