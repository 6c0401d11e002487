"""Multi-process (gloo, world_size 2, CPU) tests of the distributed paths:
job sharding + score all-gather of the CGNN engine, and the row-partitioned GCN."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, min(2, 8 // world)))


def _score_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.engine.program import program_for_pair
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.philox import model_key
    from cgnn_amd.utils.settings import RunConfig
    rng = np.random.default_rng(0)
    jobs = []
    for r in range(5):
        d = rng.normal(size=(2, 60)).astype(np.float32)
        jobs.append(Job(program_for_pair(8), d, model_key(1, r)))
    cfg = RunConfig(gpu=False, train_epochs=3, test_epochs=2, h_layer_dim=8)
    s = score_jobs(jobs, cfg)
    out[rank] = s.tolist()
    dist.barrier()
    dist.destroy_process_group()


def test_score_jobs_sharded_equals_single_process():
    from cgnn_amd.engine.program import program_for_pair
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.philox import model_key
    from cgnn_amd.utils.settings import RunConfig
    rng = np.random.default_rng(0)
    jobs = [Job(program_for_pair(8), rng.normal(size=(2, 60)).astype(np.float32), model_key(1, r))
            for r in range(5)]
    cfg = RunConfig(gpu=False, train_epochs=3, test_epochs=2, h_layer_dim=8)
    single = score_jobs(jobs, cfg)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_score_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_allclose(out[r], single, rtol=1e-12)   # same noise: exact


def _strip_train(g, world):
    """No train rows in the last rank's block (they become validation rows)."""
    lo = (g.n + world - 1) // world * (world - 1)
    m = g.mask[lo:]
    m[m == 1] = 2
    return g


def _gcn_worker(rank, world, port, out, halo=None, strip=False, kw=None):
    _init(rank, world, port)
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    kw = kw or {}
    g = synthetic("ogbn-products", seed=0, scale=0.002)
    if strip:
        _strip_train(g, world)
    tr = GCNTrainer(g, hidden=64, halo=halo, **kw)
    assert tr.halo == (halo if halo is not None else world >= 4)
    if tr._l2 is not None:
        assert (tr._l2.plan is not None) == kw.get("train_halo", True)
    tr.train_step()
    p1 = tr.params.clone().numpy().tolist()
    for _ in range(3):
        tr.train_step()
    res = tr.evaluate()
    out[rank] = (res, tr.params.clone().numpy().tolist(), p1)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,halo,overlap,all_rows,train_halo", [
    (2, False, "0", "0", "0"), (2, True, "0", "0", "0"), (4, None, "0", "0", "0"), (2, False, "1", "0", "1"),
    (4, None, "1", "0", "1"), (2, True, "1", "1", "1"), (4, None, "1", "1", "1"), (3, True, "1", "0", "1"),
    (3, None, "1", "0", "strip"), (8, None, "1", "0", "1"), (8, None, "1", "0", "strip")])
def test_gcn_row_partition_matches_single_process(world, halo, overlap, all_rows, train_halo):
    """Row-partitioned GCN over gloo ranks == one process; layer-2 rows of other
    ranks by all-gather or by the halo all-to-all (the default from 4 ranks); the
    backward's compact-gradient all-gather blocking or overlapped with the local edges
    (bwd_overlap); training layer 2 over the train rows only (default) or over every
    row (train_rows_only=False, against the one-process train-row run); the training
    epochs' own halo of the train rows' sources (train_halo); "strip": the last rank
    owns no train row (it joins the training halo with a placeholder)."""
    strip = train_halo == "strip"
    if strip:
        train_halo = "1"
    kw = dict(bwd_overlap=overlap == "1", train_rows_only=all_rows == "0", train_halo=train_halo == "1")
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    g = synthetic("ogbn-products", seed=0, scale=0.002)
    if strip:
        _strip_train(g, world)
    tr = GCNTrainer(g, hidden=64, rank=0, world=1)
    assert tr._l2 is not None
    tr.train_step()
    p1 = tr.params.clone().numpy()
    for _ in range(3):
        tr.train_step()
    ref = tr.evaluate()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gcn_worker, args=(world, _free_port(), out, halo, strip, kw), nprocs=world, join=True)
    for r in range(world):
        res, params, q1 = out[r]
        # after one step the partitioned run equals the single-process one up to the
        # summation order of the split gradients (bf16 activations, fp32 sums)
        np.testing.assert_allclose(np.array(q1), p1, atol=2e-3)
        assert abs(res["train_loss"] - ref["train_loss"]) < 0.02 * ref["train_loss"]
        assert abs(res["val_acc"] - ref["val_acc"]) < 0.06
    # the ranks hold bitwise-identical replicated parameters
    for r in range(1, world):
        np.testing.assert_array_equal(out[0][1], out[r][1])


def test_gcn_train_row_layer2_matches_all_rows():
    """Training epochs that aggregate layer 2 only at the train rows give the same
    losses and parameters as aggregating every row (one process)."""
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    g = synthetic("ogbn-products", seed=1, scale=0.002)
    runs = []
    for rows_only in (False, True):
        tr = GCNTrainer(g, hidden=64, rank=0, world=1, train_rows_only=rows_only)
        assert (tr._l2 is None) == (not rows_only)
        losses = []
        for _ in range(4):
            tr.train_step()
            losses.append(tr.train_loss())
        runs.append((losses, tr.params.clone(), tr.evaluate()))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-5)
    torch.testing.assert_close(runs[1][1], runs[0][1], rtol=1e-4, atol=1e-5)
    assert runs[1][2] == pytest.approx(runs[0][2], rel=1e-4, abs=1e-4)


def _mmd_data():
    g = torch.Generator().manual_seed(3)
    pred = torch.randn(2, 60, 3, generator=g, dtype=torch.float64)
    true = torch.randn(2, 60, 3, generator=g, dtype=torch.float64) * 1.3 + 0.2
    return pred, true


def _mmd_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.parallel.sharded_mmd import mmd_loss_sharded
    pred, true = _mmd_data()
    lo, hi = (0, 37) if rank == 0 else (37, 60)       # unequal shards
    p = pred[:, lo:hi].clone().requires_grad_(True)
    loss = mmd_loss_sharded(p, true[:, lo:hi])
    loss.sum().backward()
    out[rank] = (loss.detach().numpy().tolist(), p.grad.numpy().tolist())
    dist.destroy_process_group()


def test_sharded_mmd_matches_full_mmd():
    """Sample-sharded MMD over 2 gloo ranks: every rank sees the global loss and
    gets exactly its rows of the full gradient."""
    from cgnn_amd.engine.reference import mmd_loss_dense
    pred, true = _mmd_data()
    p = pred.clone().requires_grad_(True)
    ref = torch.stack([mmd_loss_dense(p[r], true[r]) for r in range(2)])
    ref.sum().backward()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_mmd_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for rank, (lo, hi) in enumerate([(0, 37), (37, 60)]):
        loss, grad = out[rank]
        np.testing.assert_allclose(loss, ref.detach().numpy(), rtol=1e-10)
        np.testing.assert_allclose(np.array(grad), p.grad[:, lo:hi].numpy(), rtol=1e-8, atol=1e-12)


def _bucket_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.parallel.ddp import GradBucketer
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    # tiny buckets: several collectives, launched from the backward hooks
    ddp = GradBucketer(list(model.parameters()), bucket_mb=60 * 4 / 2 ** 20)
    assert len(ddp.buckets) > 1
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(32, 6, generator=g)
    model(x).square().mean().backward()
    local = [p.grad.clone() for p in model.parameters()]
    gathered = [[torch.zeros_like(t) for _ in range(world)] for t in local]
    for t, lst in zip(local, gathered):
        dist.all_gather(lst, t)
    ddp.finish()
    for p, lst in zip(model.parameters(), gathered):
        torch.testing.assert_close(p.grad, sum(lst) / world, rtol=1e-6, atol=1e-7)
    out[rank] = True
    dist.destroy_process_group()


def test_grad_bucketer_averages_gradients():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] and out[1]


def _sage_dp_worker(rank, world, port, out):
    _init(rank, world, port)
    torch.set_num_threads(1)
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=0, scale=0.001 if world <= 2 else 0.004)
    tr = SAGETrainer(g, hidden=32, layers=3, fanouts=(5, 4, 3), batch_size=64, seed=rank * 7, prefetch=False)
    n_batches = len(tr._batches())
    l0 = tr.train_epoch()
    l1 = tr.train_epoch()
    out[rank] = (n_batches, l0, l1, torch.cat([p.detach().flatten() for p in tr.model.parameters()]).numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sage_data_parallel_keeps_replicas_identical(world):
    """3-layer SAGE mini-batch DP over 2 and 8 gloo ranks (different init seeds are
    overwritten by rank 0's broadcast): same number of steps on every rank, and
    the averaged gradients keep the replicas bitwise identical."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sage_dp_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert all(out[r][0] == out[0][0] > 0 for r in range(world))
    for r in range(1, world):
        np.testing.assert_array_equal(out[0][3], out[r][3])
    assert np.isfinite(out[0][1]) and np.isfinite(out[0][2])


def _gat_params(tr):
    if tr.fused is not None:
        return tr.fused.params.detach().clone().numpy()
    return torch.cat([p.detach().flatten() for p in tr.model.parameters()]).numpy()


def _gat_shard_worker(rank, world, port, out, fused=False, heads=2, dropout=0.0, chunk=4 << 30, strip=False,
                      l1_exchange=False, train_halo=True, partition="none"):
    _init(rank, world, port)
    from cgnn_amd.gnn.data import synthetic_shard
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    # rank-local generation: this rank never builds the rest of the graph (with the
    # locality partition it builds the graph's structure once to order it)
    shard = synthetic_shard("ogbn-products", rank, world, seed=1, scale=0.0005, partition=partition)
    if strip and rank == world - 1:          # this rank owns no train row
        shard.mask[shard.mask == 1] = 2
    tr = ShardedGATTrainer(shard, heads=heads, head_dim=8, dropout=dropout, lr=0.01, seed=rank, fused=fused,
                           halo_chunk_bytes=chunk, l1_exchange=l1_exchange, train_halo=train_halo)
    if chunk < (1 << 20):
        assert tr.halo.rounds > 1
    if tr.fused is not None and train_halo:
        # training epochs exchange only the train rows' sources (their own halo)
        th = tr.fused._tr.halo
        assert th is not tr.halo and th.n_recv <= tr.halo.n_recv
    losses = []
    grads1 = None
    for _ in range(3):
        l = tr.train_step().clone()
        dist.all_reduce(l)
        losses.append(float(l))
        if grads1 is None and tr.fused is not None:
            grads1 = tr.fused.grads.clone().numpy()
    res = tr.evaluate()
    out[rank] = (losses, res, _gat_params(tr), tr.halo_stats(), grads1)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk", [(2, 4 << 30), (4, 4 << 30), (4, 16 << 10)])
def test_sharded_gat_matches_single_process(world, chunk):
    """GAT with rows sharded over gloo ranks -- rank-local shard generation, halo
    all-to-all of exactly the [Wh | s_src] rows each rank reads, gradients returned
    to their owners, averaged parameter gradients -- equals the unsharded model:
    same global losses, accuracies and parameters."""
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    g = synthetic("ogbn-products", seed=1, scale=0.0005)
    ref = ShardedGATTrainer(g, heads=2, head_dim=8, dropout=0.0, lr=0.01, seed=0)
    ref_losses = [float(ref.train_step()) for _ in range(3)]
    ref_res = ref.evaluate()
    ref_params = torch.cat([p.detach().flatten() for p in ref.model.parameters()]).numpy()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gat_shard_worker, args=(world, _free_port(), out, False, 2, 0.0, chunk), nprocs=world, join=True)
    for r in range(world):
        losses, res, params, hs, _ = out[r]
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        assert res == pytest.approx(ref_res, abs=1e-9)
        # (summation order of the returned halo gradients differs from the unsharded sum)
        np.testing.assert_allclose(params, ref_params, rtol=1e-4, atol=3e-5)
        assert 0 < hs["recv_rows"] < g.n - hs["local_rows"] or hs["recv_rows"] == g.n - hs["local_rows"]
    assert sum(out[r][3]["recv_rows"] for r in range(world)) == sum(out[r][3]["send_rows"] for r in range(world))
    np.testing.assert_array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("world,chunk,strip,l1x", [(2, 4 << 30, False, False), (4, 4 << 30, False, False),
                                                   (2, 16 << 10, False, False), (4, 16 << 10, False, False),
                                                   (3, 4 << 30, True, False), (2, 4 << 30, False, True),
                                                   (4, 16 << 10, False, True), (8, 16 << 10, False, False)])
def test_sharded_fused_gat_matches_single_process(world, chunk, strip, l1x):
    """The fused GAT epoch (gat_fused: every dense op a HIP kernel on a GPU; its fp32
    reference branches here) sharded over gloo ranks equals the one-process fused
    model -- with dropout on, since the masks are keyed by the global row.  Training
    layer 2 runs at the train rows over a training halo; ``strip``: the last rank
    owns no train row (placeholder row in the collective plan).  Layer 1 is projected
    locally from the setup-time halo input rows (no per-epoch exchange) unless ``l1x``
    (l1_exchange=True: the per-epoch [Wh | s_src] exchange)."""
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    g = synthetic("ogbn-products", seed=1, scale=0.0005)
    if strip:
        _strip_train(g, world)
    ref = ShardedGATTrainer(g, heads=4, head_dim=8, dropout=0.3, lr=0.01, seed=0, fused=True)
    assert ref.fused is not None
    ref_losses = [float(ref.train_step())]
    ref_grads1 = ref.fused.grads.clone().numpy()
    ref_losses += [float(ref.train_step()) for _ in range(2)]
    ref_res = ref.evaluate()
    ref_params = _gat_params(ref)
    mgr = mp.Manager()
    out = mgr.dict()
    # chunk 16 KB: the halo exchanges run in several rounds (bounded staging memory)
    mp.spawn(_gat_shard_worker, args=(world, _free_port(), out, True, 4, 0.3, chunk, strip, l1x), nprocs=world,
             join=True)
    for r in range(world):
        losses, res, params, hs, grads1 = out[r]
        assert hs["layer1_local"] == (not l1x) and (hs["layer1_recv_bytes"] == 0) == (not l1x)
        # first-step gradients (rank-summed): equal up to the summation order of the
        # halo-returned rows, which are then stored bf16 as the MFMA operand
        # (a locally projected layer 1 rounds each rank's partial of a received row: 2e-3)
        tol = 1e-3 if l1x else 2e-3
        assert np.abs(grads1 - ref_grads1).max() < tol * np.abs(ref_grads1).max()
        # the gradient rows returned by the halo are summed in another order and then
        # stored bf16 (as the MFMA weight-gradient operand), so a rounding can flip
        np.testing.assert_allclose(losses, ref_losses, rtol=2e-4)
        assert res == pytest.approx(ref_res, abs=2e-3)
        # Adam normalises each gradient, so a near-zero gradient perturbed by such a
        # rounding moves its weight by up to ~lr: bound the worst element by lr / 10
        # and require (nearly) all of them to agree closely
        d = np.abs(params - ref_params)
        if l1x:
            assert d.max() < 1e-3 and np.mean(d > 1e-4) < 0.05, (d.max(), np.mean(d > 1e-4))
        else:
            # local layer 1: a received row's share of its [dWh | ds_src] gradient is stored
            # bf16 on the rank that made it (the weight-gradient operand) instead of being
            # summed at the owner first -- one more bf16 rounding per partial, so Adam's
            # per-element normalisation moves more weights by ~1e-4 (and a sign flip of a
            # near-zero gradient by up to 2 lr)
            assert d.max() < 2.5e-2 and np.mean(d > 1e-3) < 0.02, (d.max(), np.mean(d > 1e-3))
    np.testing.assert_array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_fused_gat_locality_partition_matches_single_process(world):
    """Shards of the locality partition (partition_order: the reorder pass over the
    graph's structure, computed by every rank on its own) train like the one-process
    model of the reordered graph."""
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    g, _ = reorder(synthetic("ogbn-products", seed=1, scale=0.0005), seed=1)
    ref = ShardedGATTrainer(g, heads=4, head_dim=8, dropout=0.3, lr=0.01, seed=0, fused=True)
    ref_losses = [float(ref.train_step()) for _ in range(3)]
    ref_res = ref.evaluate()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gat_shard_worker, args=(world, _free_port(), out, True, 4, 0.3, 4 << 30, False, False, True,
                                      "locality"), nprocs=world, join=True)
    for r in range(world):
        losses, res, params, hs, _ = out[r]
        np.testing.assert_allclose(losses, ref_losses, rtol=5e-4)
        # (the split gradients' summation order may flip one near-tie prediction of ~100)
        assert res == pytest.approx(ref_res, abs=0.011)
    np.testing.assert_array_equal(out[0][2], out[1][2])


def test_sharded_fused_gat_without_train_halo_rank_without_train_rows():
    """train_halo=False with a rank that owns no train row: the train-neighbour flag
    exchange must still run on every rank (a per-rank decision around a collective would
    pair that rank's first training exchange with its peers' flag exchange)."""
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    world = 3
    g = synthetic("ogbn-products", seed=1, scale=0.0005)
    _strip_train(g, world)
    ref = ShardedGATTrainer(g, heads=4, head_dim=8, dropout=0.3, lr=0.01, seed=0, fused=True)
    ref_losses = [float(ref.train_step()) for _ in range(3)]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gat_shard_worker, args=(world, _free_port(), out, True, 4, 0.3, 4 << 30, True, False, False),
             nprocs=world, join=True)
    for r in range(world):
        np.testing.assert_allclose(out[r][0], ref_losses, rtol=5e-4)


@pytest.mark.parametrize("halo", [False, True])
def test_gcn_forced_collectives_one_rank_equals_plain(halo):
    """GCNTrainer(collectives=True) on a 1-rank group takes every multi-rank branch
    (exchanges, split aggregation, gradient all-reduce) and reproduces the plain trainer
    (the GPU variant of this test runs the same over RCCL, tests/test_rccl_gpu.py)."""
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        g = synthetic("ogbn-products", seed=2, scale=0.001)
        ref = GCNTrainer(g, hidden=64, rank=0, world=1)
        forced = GCNTrainer(g, hidden=64, rank=0, world=1, collectives=True, halo=halo)
        assert forced.multi and not ref.multi and forced.halo == halo
        for _ in range(3):
            ref.train_step()
            forced.train_step()
        assert abs(ref.train_loss() - forced.train_loss()) < 1e-4 * ref.train_loss()
        np.testing.assert_allclose(forced.params.numpy(), ref.params.numpy(), atol=1e-4, rtol=0)
        assert ref.evaluate() == pytest.approx(forced.evaluate(), abs=2e-3)
    finally:
        dist.destroy_process_group()


def _selftest_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.parallel.collectives import selftest
    out[rank] = selftest("cpu")
    dist.destroy_process_group()


def test_collectives_selftest_gloo_two_ranks():
    """bench.py gates every multi-rank run on collectives.selftest(): its gloo branch
    (host tensors, list-form all_gather) passes on 2 ranks and reports the group."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_selftest_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert out[r]["backend"] == "gloo" and out[r]["world_size"] == 2, out[r]


def _order_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.gnn import data
    calls = []
    real = data.partition_order

    def counted(*a, **k):
        calls.append(rank)
        return real(*a, **k)

    data.partition_order = counted
    order = data.shared_partition_order("ogbn-products", seed=3, scale=0.002)
    out[rank] = (order, list(calls))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shared_partition_order_runs_once_and_broadcasts(world):
    """The papers100M locality partition is computed by rank 0 only and broadcast
    (every rank recomputed the whole 111 M-node pass): every rank gets
    the one-process order."""
    from cgnn_amd.gnn.data import partition_order
    ref = partition_order("ogbn-products", seed=3, scale=0.002)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_order_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        np.testing.assert_array_equal(out[r][0], ref)
        assert out[r][1] == ([0] if r == 0 else [])


def _order_fail_worker(rank, world, port, out):
    _init(rank, world, port)
    from cgnn_amd.gnn import data

    def broken(*a, **k):
        raise MemoryError("partition pass failed on rank 0")

    data.partition_order = broken
    try:
        data.shared_partition_order("ogbn-products", seed=3, scale=0.002)
        out[rank] = "returned"
    except MemoryError:
        out[rank] = "MemoryError"
    except RuntimeError as e:
        out[rank] = "RuntimeError: " + str(e)[:60]
    dist.destroy_process_group()


def test_shared_partition_order_failure_raises_on_every_rank():
    """a pass that raises on rank 0 makes every rank raise (status word ahead
    of the broadcast) instead of leaving the other ranks blocked in the collective."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_order_fail_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert out[0] == "MemoryError"
    for r in (1, 2):
        assert out[r].startswith("RuntimeError: broadcast_host_array: source rank 0"), out[r]
