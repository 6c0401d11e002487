"""HIP kernels of the CGNN engine vs the PyTorch fp64 oracle (engine/reference.py)."""
import numpy as np
import pytest
import torch

from cgnn_amd import native
from cgnn_amd.engine.batch import DeviceTrainer, mmd_geometry, padded_dim
from cgnn_amd.engine.program import program_for_confounders, program_for_dag, program_for_pair
from cgnn_amd.engine.reference import ReferenceTrainer, mmd_loss_dense
from cgnn_amd.utils.graph import DirectedGraph, UndirectedGraph
from cgnn_amd.utils.philox import model_key

pytestmark = pytest.mark.gpu


def test_native_extension_is_loaded():
    hip = native.hip()
    assert hip.device_count() >= 1
    assert hip.__file__.startswith(__import__("os").path.dirname(native.__file__))


@pytest.mark.parametrize("N,d,kernel", [(2, 1, "valu"), (63, 2, "valu"), (64, 5, "valu"), (257, 22, "valu"),
                                        (1000, 22, "valu"), (1500, 2, "valu"), (700, 1, "valu"), (600, 4, "valu"),
                                        (513, 6, "valu"), (800, 8, "valu"), (33, 8, "mfma"),
                                        (257, 22, "mfma"), (1000, 22, "mfma"), (500, 40, "mfma"),
                                        (130, 64, "mfma")])
def test_mmd_loss_and_grad_match_oracle(N, d, kernel):
    from cgnn_amd.ops.mmd import mmd_loss
    torch.manual_seed(N * 7 + d)
    R = 3
    pred = torch.randn(R, N, d, dtype=torch.float64)
    true = torch.randn(R, N, d, dtype=torch.float64) * 1.3 + 0.2
    # oracle
    ref_l, ref_g = [], []
    for r in range(R):
        p = pred[r].clone().requires_grad_(True)
        L = mmd_loss_dense(p, true[r])
        (g,) = torch.autograd.grad(L, p)
        ref_l.append(float(L))
        ref_g.append(g)
    pg = pred.float().cuda().requires_grad_(True)
    out = mmd_loss(pg, true.float().cuda(), kernel=kernel)
    out.sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref_l, rtol=2e-4, atol=2e-5)
    gref = torch.stack(ref_g).numpy()
    scale = np.abs(gref).max()
    np.testing.assert_allclose(pg.grad.cpu().numpy(), gref, rtol=2e-3, atol=2e-3 * scale)


@pytest.mark.parametrize("N,d", [(1500, 2), (513, 6), (800, 8)])
def test_mmd_symmetric_training_matches_full_block(N, d):
    """The mirrored pred-pred evaluation (off-diagonal tiles once, column sums by the
    staggered DPP rotation) equals the full-block kernel to fp32 rounding, and the
    symmetric launch really adds its mirror slots."""
    from cgnn_amd.engine.batch import mmd_mirror_slots
    from cgnn_amd.ops.mmd import mmd_loss
    assert mmd_mirror_slots(padded_dim(d), N) == (N + 255) // 256 - 1
    torch.manual_seed(N + d)
    pred = torch.randn(4, N, d, device="cuda")
    true = torch.randn(4, N, d, device="cuda") * 0.8 - 0.3
    outs = []
    for sym in (True, False):
        p = pred.clone().requires_grad_(True)
        L = mmd_loss(p, true, kernel="valu", symmetric=sym)
        L.sum().backward()
        outs.append((L.detach(), p.grad))
    (l1, g1), (l0, g0) = outs
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-4 * float(g0.abs().max()))


def _toy_dag():
    g = DirectedGraph()
    for a, b in [("A", "B"), ("A", "C"), ("B", "D"), ("C", "D"), ("D", "E")]:
        g.add(a, b)
    return g


def _data(d, N, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((d, N)).astype(np.float32)
    x[1] += 0.8 * x[0]
    return x


@pytest.mark.parametrize("kind", ["pair", "dag", "conf"])
@pytest.mark.parametrize("fast", [False, True])
def test_device_trainer_matches_oracle(kind, fast):
    H = 20
    if kind == "pair":
        progs = [program_for_pair(H)] * 3
        d = 2
    elif kind == "dag":
        g = _toy_dag()
        progs = [program_for_dag(g, H)] * 3
        d = 5
    else:
        g = _toy_dag()
        skel = UndirectedGraph()
        for a, b, _ in g.get_list_edges():
            skel.add(a, b)
        skel.add("B", "C")
        dg = DirectedGraph(skeleton=skel)
        for a, b, _ in g.get_list_edges():
            dg.add(a, b)
        progs = [program_for_confounders(dg, H)] * 3
        d = 5
    N = 300
    datas = [_data(d, N, s) for s in range(3)]
    keys = [model_key(7, kind, r) for r in range(3)]
    kw = dict(learning_rate=0.01, init_std=0.05, use_fast_mmd=fast, nb_vectors=20)
    ref = ReferenceTrainer(progs, datas, keys, H, **kw)
    ref_scores = ref.run(6, 4)
    dev = DeviceTrainer(progs, datas, keys, H, "cuda:0", record_history=6, graph_chunk=3, **kw)
    scores = dev.run(6, 4)
    hist = dev.history()
    np.testing.assert_allclose(hist, np.array(ref.loss_history), rtol=3e-3, atol=1e-5)
    np.testing.assert_allclose(scores, ref_scores, rtol=3e-3, atol=1e-5)


def test_mfma_and_vector_mmd_trainers_agree():
    """A 10-variable DAG (padded D = 12) trained with the matrix-core MMD and with
    the vector MMD: the two differ only by the distance formula's rounding."""
    H = 16
    g = DirectedGraph()
    for k in range(9):
        g.add("V%d" % k, "V%d" % (k + 1))
    g.add("V0", "V5")
    prog = program_for_dag(g, H)
    N = 400
    datas = [_data(10, N, s) for s in range(3)]
    keys = [model_key(5, "mf", r) for r in range(3)]
    a = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0", record_history=8, mmd_kernel="mfma")
    b = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0", record_history=8, mmd_kernel="valu")
    assert a.mmd_kernel == "mfma" and b.mmd_kernel == "valu"
    sa, sb = a.run(8, 4), b.run(8, 4)
    np.testing.assert_allclose(a.history(), b.history(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(sa, sb, rtol=1e-4, atol=1e-6)
    # without a recorded history the training steps skip the (unread) loss:
    # same gradients, same scores
    c = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0", mmd_kernel="mfma").run(8, 4)
    np.testing.assert_allclose(c, sa, rtol=1e-6)
    ref = ReferenceTrainer([prog] * 3, datas, keys, H)
    np.testing.assert_allclose(sa, ref.run(8, 4), rtol=3e-3, atol=1e-5)


def test_graph_replay_equals_eager():
    H = 20
    g = _toy_dag()
    progs = [program_for_dag(g, H)] * 2
    datas = [_data(5, 200, s) for s in range(2)]
    keys = [model_key(3, "x", r) for r in range(2)]
    a = DeviceTrainer(progs, datas, keys, H, "cuda:0", graph_chunk=0).run(20, 10)
    b = DeviceTrainer(progs, datas, keys, H, "cuda:0", graph_chunk=7).run(20, 10)
    np.testing.assert_array_equal(a, b)   # bitwise: deterministic reductions, no atomics


def test_verbose_object_api_logs_without_changing_the_score(capsys):
    """CGNN_model on the GPU: verbose train/evaluate print iterations 0, 100, ... (the
    recorded history; the chunked evaluation reads loss_last), and the score is bitwise
    the silent run's."""
    from cgnn_amd.models.cgnn import CGNN_model
    g = _toy_dag()
    data = _data(5, 300, 1).T
    kw = dict(train_epochs=230, test_epochs=120, h_layer_dim=20, gpu=True, nb_gpu=1)
    a = CGNN_model(300, g, run=1, idx=2, **kw)
    a.train(data, verbose=True)
    sa = a.evaluate(data, verbose=True)
    lines = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Pair:")]
    assert [int(l.split("Iter:")[1].split(",")[0]) for l in lines] == [0, 100, 200, 0, 100]
    b = CGNN_model(300, g, run=1, idx=2, **kw)
    b.train(data, verbose=False)
    sb = b.evaluate(data, verbose=False)
    assert capsys.readouterr().out.count("Pair:") == 0
    assert sa == sb


def test_batch_composition_does_not_change_scores():
    H = 20
    g = _toy_dag()
    prog = program_for_dag(g, H)
    datas = [_data(5, 600, s) for s in range(4)]      # 3 row tiles: the symmetric MMD's mirror slots
    keys = [model_key(11, "y", r) for r in range(4)]
    full = DeviceTrainer([prog] * 4, datas, keys, H, "cuda:0").run(10, 5)
    for r in range(4):
        one = DeviceTrainer([prog], [datas[r]], [keys[r]], H, "cuda:0").run(10, 5)
        # bitwise: kernel geometry and summation orders never depend on the batch size,
        # so a score is identical on 1 or 8 GPUs / in any batch
        np.testing.assert_array_equal(one, full[r:r + 1])


def test_batch_composition_bitwise_wide_joint():
    """Same for the matrix-core MMD path (d = 10 -> D = 12)."""
    H = 16
    g = DirectedGraph()
    for k in range(9):
        g.add("V%d" % k, "V%d" % (k + 1))
    prog = program_for_dag(g, H)
    datas = [_data(10, 333, s) for s in range(3)]
    keys = [model_key(12, "w", r) for r in range(3)]
    full = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0").run(6, 3)
    one = DeviceTrainer([prog], [datas[2]], [keys[2]], H, "cuda:0").run(6, 3)
    np.testing.assert_array_equal(one, full[2:3])


@pytest.mark.parametrize("d,kernel", [(3, "valu"), (20, "valu"), (20, "mfma")])
def test_row_range_mmd_tiles_the_full_mmd(d, kernel):
    """Sample-sharded MMD building block: row ranges [b, b+n) of the HIP kernels
    against all columns sum to the full loss and give exactly those rows of the
    full gradient (parallel/sharded_mmd.py)."""
    from cgnn_amd.parallel.sharded_mmd import row_partials
    g = torch.Generator().manual_seed(5)
    R, N = 3, 700
    pred = torch.randn(R, N, d, generator=g, dtype=torch.float64)
    true = torch.randn(R, N, d, generator=g, dtype=torch.float64) * 1.2 + 0.1
    p = pred.clone().requires_grad_(True)
    ref = torch.stack([mmd_loss_dense(p[r], true[r]) for r in range(R)])
    ref.sum().backward()
    P, T = pred.float().cuda(), true.float().cuda()
    total = torch.zeros(R, dtype=torch.float64)
    for b, e in [(0, 300), (300, 513), (513, 700)]:
        loss, grad = row_partials(P[:, b:e], T[:, b:e], P, T, b, kernel)
        total += loss.double().cpu()
        np.testing.assert_allclose(grad.double().cpu().numpy(), p.grad[:, b:e].numpy(), rtol=2e-3, atol=2e-7)
    np.testing.assert_allclose((total / N**2).numpy(), ref.detach().numpy(), rtol=2e-4, atol=1e-7)


def test_rff_matrix_core_matches_oracle():
    """Fast MMD (random Fourier features) on the exact-fp32 matrix cores vs the fp64
    oracle, on a 10-variable DAG (padded D = 12) and a pair."""
    H = 16
    g = DirectedGraph()
    for k in range(9):
        g.add("V%d" % k, "V%d" % (k + 1))
    for prog, d in ((program_for_dag(g, H), 10), (program_for_pair(H), 2)):
        N = 350
        datas = [_data(d, N, s) for s in range(3)]
        keys = [model_key(11, "rff", r) for r in range(3)]
        kw = dict(learning_rate=0.01, init_std=0.05, use_fast_mmd=True, nb_vectors=30)
        ref = ReferenceTrainer([prog] * 3, datas, keys, H, **kw)
        ref_scores = ref.run(6, 4)
        a = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0", record_history=6, **kw)
        sa = a.run(6, 4)
        np.testing.assert_allclose(a.history(), np.array(ref.loss_history), rtol=3e-3, atol=1e-5)
        np.testing.assert_allclose(sa, ref_scores, rtol=3e-3, atol=1e-5)


@pytest.mark.parametrize("D", [2, 12, 64])
def test_rff_matrix_core_equals_vector_kernels(D):
    """The matrix-core and the vector Fourier-feature kernels on the same draws: same
    loss partials and gradient up to summation order."""
    hip = native.hip()
    R, N, k = 3, 333, 30
    F = 7 * k
    torch.manual_seed(D)
    xhat = torch.randn(R, D, N, device="cuda") * 0.7
    data = torch.randn(R, D, N, device="cuda") * 0.7 + 0.1
    keys = torch.randint(0, 2**31 - 1, (R, 2), dtype=torch.int32, device="cuda")
    step = torch.zeros(2, dtype=torch.int32, device="cuda")
    W = torch.zeros(R, F, D + 1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    hip.rff_freqs(W.data_ptr(), keys.data_ptr(), step.data_ptr(), 0, k, D, 7, D, R, st)
    outs = []
    for force in (0, 1):
        diff = torch.zeros(R, F, device="cuda")
        lp = torch.zeros(R, (F + 255) // 256, device="cuda")
        gp = torch.zeros(1, R, D, N, device="cuda")
        hip.rff_fwd_bwd(0, xhat.data_ptr(), data.data_ptr(), W.data_ptr(), diff.data_ptr(), lp.data_ptr(),
                        gp.data_ptr(), N, D, F, R, k, (2.0 / k) ** 0.5, st, force_valu=force)
        outs.append((lp.sum(1), gp))
    torch.cuda.synchronize()
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=1e-6)
    g = outs[1][1]
    torch.testing.assert_close(outs[0][1], g, rtol=1e-3, atol=1e-4 * float(g.abs().max()))


def test_sample_sharded_trainer_gpu_matches_oracle_and_engine():
    """The long-N trainer (engine/sharded.py) on the HIP kernels, one rank: equals the
    fp64 oracle and the hipGraph engine (DeviceTrainer) on the same job."""
    from cgnn_amd.engine.sharded import SampleShardedTrainer
    H = 16
    g = DirectedGraph()
    for k in range(9):
        g.add("V%d" % k, "V%d" % (k + 1))
    for prog, d in ((program_for_pair(H), 2), (program_for_dag(g, H), 10)):
        N = 512
        data = _data(d, N, 4)
        key = [model_key(9, "long", 0)]
        ref = ReferenceTrainer([prog], [data], key, H).run(5, 3)
        sh = SampleShardedTrainer([prog], [data], key, H, "cuda:0", N).run(5, 3)
        eng = DeviceTrainer([prog], [data], key, H, "cuda:0").run(5, 3)
        np.testing.assert_allclose(sh, ref, rtol=3e-3, atol=1e-5)
        np.testing.assert_allclose(sh, eng, rtol=1e-4, atol=1e-6)


def test_in_process_multi_device_round_robin_matches_one_device():
    """score_jobs' in-process multi-GPU path (batches round-robin over the devices of
    one process, a bounded window of in-flight batches per device) -- exercised on one
    MI355X by listing it twice (device_ids=(0, 0)): more batches than the in-flight
    window, scores bitwise equal to one device and to the per-batch ordering."""
    from cgnn_amd.engine.program import program_for_pair
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.settings import RunConfig
    rng = np.random.default_rng(7)
    jobs = [Job(program_for_pair(8), rng.normal(size=(2, 200)).astype(np.float32), model_key(3, r))
            for r in range(22)]
    base = dict(gpu=True, train_epochs=12, test_epochs=5, h_layer_dim=8, batch_models=2)
    one = score_jobs(jobs, RunConfig(device_ids=(0,), **base))          # 11 batches, window 4
    two = score_jobs(jobs, RunConfig(device_ids=(0, 0), **base))        # 11 batches, window 8
    big = score_jobs(jobs, RunConfig(device_ids=(0,), **dict(base, batch_models=64)))
    assert np.all(np.isfinite(one))
    np.testing.assert_array_equal(one, two)
    np.testing.assert_array_equal(one, big)


def test_multi_device_graph_search_matches_one_device():
    """The reference's multi-GPU placement for the graph workload (run_CGNN_graph.py:7
    sets NB_GPU = 2; runs go round-robin to /gpu:(run % NB_GPU), CGNN.py:187-188): the
    public CGNN hill climbing with batches dealt over two device entries (device_ids
    (0, 0): two streams on one MI355X) returns the same graph and scores as one device."""
    import pandas as pd
    import cgnn
    rng = np.random.default_rng(11)
    n = 300
    a = rng.normal(size=n)
    b = np.tanh(a) + 0.3 * rng.normal(size=n)
    c = b ** 2 + 0.3 * rng.normal(size=n)
    d = a - c + 0.3 * rng.normal(size=n)
    df = pd.DataFrame({"A": a, "B": b, "C": c, "D": d})
    dag = DirectedGraph()
    for u, v, w in (("B", "A", 0.1), ("B", "C", 0.2), ("D", "C", 0.3), ("A", "D", 0.4)):
        dag.add(u, v, w)
    kw = dict(nb_runs=6, train_epochs=20, test_epochs=10, h_layer_dim=8, batch_models=2, gpu=True, seed=5)
    m = cgnn.CGNN(backend="TensorFlow")
    one = m.orient_directed_graph(df, dag, device_ids=(0,), **kw)
    two = m.orient_directed_graph(df, dag, device_ids=(0, 0), **kw)
    assert sorted(one.get_list_edges()) == sorted(two.get_list_edges())


def _shared_gpu_score_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.settings import RunConfig
    rng = np.random.default_rng(9)
    jobs = [Job(program_for_pair(8), rng.normal(size=(2, 150)).astype(np.float32), model_key(4, r))
            for r in range(7)]
    g = DirectedGraph()
    for u, v in (("V0", "V1"), ("V1", "V2"), ("V0", "V3")):
        g.add(u, v)
    jobs += [Job(program_for_dag(g, 8), rng.normal(size=(4, 150)).astype(np.float32), model_key(5, r))
             for r in range(5)]
    out[rank] = score_jobs(jobs, RunConfig(gpu=True, train_epochs=10, test_epochs=4, h_layer_dim=8,
                                           batch_models=3)).tolist()
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_sharing_the_gpu_score_like_one_process():
    """One process per GPU (torchrun) shards the jobs by index over the ranks and
    all-gathers the scores (parallel/dist.py): 2 gloo ranks sharing cuda:0 give every
    rank the one-process scores, pairwise and graph jobs alike, bit for bit."""
    import socket
    import torch.multiprocessing as mp
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.settings import RunConfig
    rng = np.random.default_rng(9)
    jobs = [Job(program_for_pair(8), rng.normal(size=(2, 150)).astype(np.float32), model_key(4, r))
            for r in range(7)]
    g = DirectedGraph()
    for u, v in (("V0", "V1"), ("V1", "V2"), ("V0", "V3")):
        g.add(u, v)
    jobs += [Job(program_for_dag(g, 8), rng.normal(size=(4, 150)).astype(np.float32), model_key(5, r))
             for r in range(5)]
    single = score_jobs(jobs, RunConfig(gpu=True, train_epochs=10, test_epochs=4, h_layer_dim=8, batch_models=3))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_shared_gpu_score_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    assert np.all(np.isfinite(single))
    for r in range(2):
        np.testing.assert_array_equal(np.array(out[r]), single)


@pytest.mark.parametrize("D", [12, 64, 256])
def test_rff_wide_form_equals_narrow(D):
    """The wide Fourier-feature form (theta scratch image; the only one above D = 256)
    against the register forms on the same draws: same loss partials and gradient up to
    summation order."""
    hip = native.hip()
    R, N, k = 2, 301, 40
    F = 7 * k
    torch.manual_seed(D + 1)
    xhat = torch.randn(R, D, N, device="cuda") * 0.5
    data = torch.randn(R, D, N, device="cuda") * 0.5 + 0.1
    keys = torch.randint(0, 2**31 - 1, (R, 2), dtype=torch.int32, device="cuda")
    step = torch.zeros(2, dtype=torch.int32, device="cuda")
    W = torch.zeros(R, F, D + 1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    hip.rff_freqs(W.data_ptr(), keys.data_ptr(), step.data_ptr(), 0, k, D, 7, D, R, st)
    scratch = torch.zeros(hip.rff_wide_scratch_floats(N, F, R), device="cuda")
    outs = []
    for wide in (0, 1):
        diff = torch.zeros(R, F, device="cuda")
        lp = torch.zeros(R, (F + 255) // 256, device="cuda")
        gp = torch.zeros(1, R, D, N, device="cuda")
        hip.rff_fwd_bwd(0, xhat.data_ptr(), data.data_ptr(), W.data_ptr(), diff.data_ptr(), lp.data_ptr(),
                        gp.data_ptr(), N, D, F, R, k, (2.0 / k) ** 0.5, st, scratch=scratch.data_ptr(),
                        force_wide=wide)
        outs.append((lp.sum(1), diff, gp))
    torch.cuda.synchronize()
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-4, atol=1e-7)
    g = outs[0][2]
    torch.testing.assert_close(outs[1][2], g, rtol=1e-3, atol=1e-4 * float(g.abs().max()))
