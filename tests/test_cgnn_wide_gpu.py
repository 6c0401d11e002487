"""CGNN beyond the narrow shapes: causal graphs with more than 64 variables and any
``h_layer_dim`` (the reference builds one MLP per node for any d and h,
/root/reference/Code/cgnn/CGNN.py:63-90; its generator defaults to 200 variables,
generators/random_graph_generator.py:26).  Device trainers vs the fp64 oracle."""
import numpy as np
import pytest
import torch

from cgnn_amd import native
from cgnn_amd.engine.batch import DeviceTrainer, device_supported, padded_dim
from cgnn_amd.engine.program import program_for_dag
from cgnn_amd.engine.reference import ReferenceTrainer, mmd_loss_dense
from cgnn_amd.utils.graph import DirectedGraph
from cgnn_amd.utils.philox import model_key

pytestmark = pytest.mark.gpu


def _random_dag(d, seed, max_par=3):
    rng = np.random.default_rng(seed)
    g = DirectedGraph()
    names = ["V%d" % k for k in range(d)]
    for k in range(1, d):
        for p in rng.choice(k, size=min(k, int(rng.integers(1, max_par + 1))), replace=False):
            g.add(names[int(p)], names[k])
    return g


def _data(d, N, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((d, N)).astype(np.float32)
    x[1:] += 0.5 * x[:-1]
    return x


@pytest.mark.parametrize("N,d", [(300, 100), (130, 200), (97, 256), (150, 300), (100, 512), (70, 1000)])
def test_wide_mmd_matches_oracle(N, d):
    from cgnn_amd.ops.mmd import mmd_loss
    torch.manual_seed(d)
    R = 2
    pred = torch.randn(R, N, d, dtype=torch.float64) * 0.3
    true = torch.randn(R, N, d, dtype=torch.float64) * 0.3 + 0.05
    ref_l, ref_g = [], []
    for r in range(R):
        p = pred[r].clone().requires_grad_(True)
        L = mmd_loss_dense(p, true[r])
        (g,) = torch.autograd.grad(L, p)
        ref_l.append(float(L))
        ref_g.append(g)
    pg = pred.float().cuda().requires_grad_(True)
    out = mmd_loss(pg, true.float().cuda(), kernel="auto")
    out.sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref_l, rtol=5e-4, atol=5e-5)
    gref = torch.stack(ref_g).numpy()
    np.testing.assert_allclose(pg.grad.cpu().numpy(), gref, rtol=3e-3, atol=3e-3 * np.abs(gref).max())


@pytest.mark.parametrize("d,H", [(100, 25), (100, 100), (200, 25), (200, 100), (300, 20), (512, 20)])
def test_wide_dag_trainer_matches_oracle(d, H):
    g = _random_dag(d, seed=d + H)
    prog = program_for_dag(g, H)
    assert padded_dim(d) > 64 and device_supported(d, H, prog.max_in)
    N = 160
    datas = [_data(d, N, s) for s in range(2)]
    keys = [model_key(13, "wide", r) for r in range(2)]
    ref = ReferenceTrainer([prog] * 2, datas, keys, H)
    ref_scores = ref.run(4, 2)
    dev = DeviceTrainer([prog] * 2, datas, keys, H, "cuda:0", record_history=4, graph_chunk=2)
    assert dev.mmd_kernel == "mfma"
    scores = dev.run(4, 2)
    np.testing.assert_allclose(dev.history(), np.array(ref.loss_history), rtol=3e-3, atol=1e-5)
    np.testing.assert_allclose(scores, ref_scores, rtol=3e-3, atol=1e-5)


@pytest.mark.parametrize("H", [7, 25, 100])
def test_generic_width_backward_small_graph_matches_oracle(H):
    """A hidden width with no compiled generator kernel on a narrow graph."""
    g = DirectedGraph()
    for a, b in [("A", "B"), ("A", "C"), ("B", "D"), ("C", "D")]:
        g.add(a, b)
    prog = program_for_dag(g, H)
    datas = [_data(4, 200, s) for s in range(3)]
    keys = [model_key(2, "h", r) for r in range(3)]
    ref = ReferenceTrainer([prog] * 3, datas, keys, H).run(5, 3)
    got = DeviceTrainer([prog] * 3, datas, keys, H, "cuda:0").run(5, 3)
    np.testing.assert_allclose(got, ref, rtol=3e-3, atol=1e-5)


def test_staged_forward_bitwise_equals_per_sample():
    """The level-scheduled forward evaluates every node with the per-sample kernel's
    fmaf order, and the noise kernel draws the same Philox normals: the generated
    samples are bitwise equal."""
    g = _random_dag(24, seed=3)                 # <= 24 variables: per-sample by default
    prog = program_for_dag(g, 20)
    datas = [_data(24, 300, s) for s in range(3)]
    keys = [model_key(4, "gb", r) for r in range(3)]
    a = DeviceTrainer([prog] * 3, datas, keys, 20, "cuda:0")
    assert a.bwd_variant == 1 and not a.staged
    a.run(0, 1)
    b = DeviceTrainer([prog] * 3, datas, keys, 20, "cuda:0", generator="staged")
    assert b.staged
    b.run(0, 1)
    np.testing.assert_array_equal(b.generated(), a.generated())
    # the squared norms too: one fmaf chain in program order in both kernels
    np.testing.assert_array_equal(b.xnorm.cpu().numpy(), a.xnorm.cpu().numpy())


def test_staged_training_matches_per_sample():
    """Same model trained by the per-sample and the level-scheduled kernels: only the
    backward's summation orders differ."""
    g = _random_dag(24, seed=4)                 # <= 24 variables: per-sample by default
    prog = program_for_dag(g, 20)
    datas = [_data(24, 257, s) for s in range(2)]
    keys = [model_key(5, "st", r) for r in range(2)]
    ta = DeviceTrainer([prog] * 2, datas, keys, 20, "cuda:0")
    assert not ta.staged
    sa = ta.run(12, 4)
    tb = DeviceTrainer([prog] * 2, datas, keys, 20, "cuda:0", generator="staged")
    assert tb.staged
    np.testing.assert_allclose(tb.run(12, 4), sa, rtol=2e-4, atol=1e-7)
    # bitwise reproducible run to run (no atomics)
    tc = DeviceTrainer([prog] * 2, datas, keys, 20, "cuda:0", generator="staged")
    np.testing.assert_array_equal(tc.run(12, 4), tb.run(12, 4))


@pytest.mark.parametrize("H", [20, 36])
def test_staged_state_placements_bitwise(H):
    """Sample state in LDS or in global memory: the same arithmetic in the same order."""
    hip = native.hip()
    d, N, R = 200, 150, 2
    g = _random_dag(d, seed=9, max_par=3)
    prog = program_for_dag(g, H)
    datas = [_data(d, N, s) for s in range(R)]
    keys = [model_key(8, "pl", r) for r in range(R)]
    tr = DeviceTrainer([prog] * R, datas, keys, H, "cuda:0")
    assert tr.staged
    tr.run(3, 1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    P, D = tr.P, tr.D
    W = 4                     # every placement fits at 4 waves per block
    outs = []
    for force in (0, 1):
        xh = torch.zeros_like(tr.xhat)
        xn = torch.zeros_like(tr.xnorm)
        hip.gen_fwd_staged(tr.prog.data_ptr(), tr.prog_stride, tr.sched.data_ptr(), tr.sched_stride,
                           tr.params.data_ptr(), P, tr.data.data_ptr(), xh.data_ptr(), tr.noise.data_ptr(), tr.NS,
                           xn.data_ptr(), N, D, d, H, tr.max_in, R, W, st, force=force)
        outs.append((xh, xn))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    torch.manual_seed(0)
    gradp = (torch.randn(2, R, D, N, device="cuda") * 1e-3).contiguous()
    T = hip.staged_tiles(N)
    grads = []
    for force in (0, 1, 2):
        gp = torch.zeros(R, T, P, device="cuda")
        dxs = torch.zeros(R, d, N, device="cuda")
        hip.gen_bwd_staged(tr.prog.data_ptr(), tr.prog_stride, tr.sched.data_ptr(), tr.sched_stride,
                           tr.params.data_ptr(), P, outs[0][0].data_ptr(), tr.noise.data_ptr(), tr.NS,
                           gradp.data_ptr(), 2, R, N, D, d, H, tr.max_in, W, gp.data_ptr(), dxs.data_ptr(), st,
                           force=force)
        grads.append(gp)
    torch.cuda.synchronize()
    assert torch.isfinite(grads[0]).all() and grads[0].abs().sum() > 0
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])


def test_wide_fourier_mmd_matches_oracle():
    g = _random_dag(90, seed=5)
    prog = program_for_dag(g, 20)
    datas = [_data(90, 150, s) for s in range(2)]
    keys = [model_key(6, "wf", r) for r in range(2)]
    kw = dict(use_fast_mmd=True, nb_vectors=40)
    ref = ReferenceTrainer([prog] * 2, datas, keys, 20, **kw).run(4, 2)
    got = DeviceTrainer([prog] * 2, datas, keys, 20, "cuda:0", **kw).run(4, 2)
    np.testing.assert_allclose(got, ref, rtol=3e-3, atol=1e-5)


def test_200_variable_generated_graph_orients_on_gpu(monkeypatch):
    """RandomGraphGenerator's default 200-variable graph through the public API on the
    GPU (short schedule: the point is the shape, not the statistics); no batch may take
    the CPU fallback."""
    import cgnn
    from cgnn_amd.engine import scorer
    from cgnn_amd.generators import RandomGraphGenerator

    def no_fallback(*a, **k):
        raise AssertionError("a 200-variable batch fell back to the CPU path")
    monkeypatch.setattr(scorer, "_run_reference", no_fallback)
    gen = RandomGraphGenerator(num_nodes=200, number_points=300, seed=0)
    graph, data = gen.generate(gen_cat=False)[:2]
    assert len(graph.get_list_nodes()) >= 200       # the last layer may overshoot (reference behaviour)
    out = cgnn.CGNN(backend="TensorFlow").orient_directed_graph(
        data, graph, nb_runs=2, train_epochs=3, test_epochs=2, h_layer_dim=20, gpu=True)
    assert isinstance(out, DirectedGraph)
    assert len(out.get_list_edges()) == len(graph.get_list_edges())
    assert not out.is_cyclic()
    assert native.hip() is not None


def test_staged_score_independent_of_batch_mates():
    """a level-scheduled batch runs W waves per block, W set by the widest
    stage of ANY program in it.  A narrow candidate scored alone (small W) and next to a
    200-wide one (W = 8) gets bit-identical losses and scores."""
    d, H, N = 200, 20, 130
    chain = DirectedGraph()
    for k in range(1, d):
        chain.add("V%d" % (k - 1), "V%d" % k)        # one node per level: W = 1
    flat = DirectedGraph()
    for k in range(1, d):
        flat.add("V0", "V%d" % k)                      # 199 nodes on one level: W = 8
    pa, pb = program_for_dag(chain, H), program_for_dag(flat, H)
    datas = [_data(d, N, s) for s in range(2)]
    keys = [model_key(21, "mates", r) for r in range(2)]
    alone = DeviceTrainer([pa], datas[:1], keys[:1], H, "cuda:0", record_history=6)
    mixed = DeviceTrainer([pa, pb], datas, keys, H, "cuda:0", record_history=6)
    assert alone.staged and mixed.staged and alone.stage_w < mixed.stage_w
    sa, sm = alone.run(6, 3), mixed.run(6, 3)
    np.testing.assert_array_equal(alone.history()[0], mixed.history()[0])
    assert sa[0] == sm[0]


@pytest.mark.parametrize("d", [300, 512])
def test_wide_fast_mmd_trainer_matches_oracle(d):
    """use_Fast_MMD beyond 256 variables (Loss.py:47-56 has no width cap; CGNN.py:92-93
    selects it for any graph): the wide Fourier-feature form trains on the GPU and matches
    the fp64 oracle."""
    H = 20
    g = _random_dag(d, seed=d + 7)
    prog = program_for_dag(g, H)
    assert device_supported(d, H, prog.max_in, len(prog.prog), fast_mmd=True)
    N = 120
    datas = [_data(d, N, s) for s in range(2)]
    keys = [model_key(17, "wrff", r) for r in range(2)]
    kw = dict(use_fast_mmd=True, nb_vectors=25)
    ref = ReferenceTrainer([prog] * 2, datas, keys, H, **kw)
    ref_scores = ref.run(4, 2)
    dev = DeviceTrainer([prog] * 2, datas, keys, H, "cuda:0", record_history=4, graph_chunk=2, **kw)
    assert dev.mmd_kernel == "rff" and dev.rff_scratch is not None
    scores = dev.run(4, 2)
    hist, ref_hist = dev.history(), np.array(ref.loss_history)
    # the first loss (same weights, same draws) to fp32 rounding; afterwards the fp32 and
    # fp64 trajectories drift apart: with ~300 inputs the projections reach ~10^3 rad
    # (frequencies 2 gamma N(0, 1), gamma up to 50), where cos / sin amplify
    # the fp32 rounding of theta into the gradient
    np.testing.assert_allclose(hist[:, 0], ref_hist[:, 0], rtol=1e-5)
    np.testing.assert_allclose(hist, ref_hist, rtol=2e-2)
    np.testing.assert_allclose(scores, ref_scores, rtol=2e-2)


def test_exact_mmd_trainer_beyond_1024_matches_oracle():
    """A 1500-variable DAG (padded 1536: the runtime-width grouped MMD) on the GPU
    against the fp64 oracle."""
    d, H, N = 1500, 8, 64
    g = _random_dag(d, seed=3, max_par=2)
    prog = program_for_dag(g, H)
    assert padded_dim(d) == 1536 and device_supported(d, H, prog.max_in, len(prog.prog))
    datas = [_data(d, N, s) for s in range(2)]
    keys = [model_key(19, "x1500", r) for r in range(2)]
    ref = ReferenceTrainer([prog] * 2, datas, keys, H)
    ref_scores = ref.run(3, 2)
    dev = DeviceTrainer([prog] * 2, datas, keys, H, "cuda:0", record_history=3, graph_chunk=0)
    assert dev.mmd_kernel == "mfma" and dev.staged
    scores = dev.run(3, 2)
    np.testing.assert_allclose(dev.history(), np.array(ref.loss_history), rtol=3e-3, atol=1e-5)
    np.testing.assert_allclose(scores, ref_scores, rtol=3e-3, atol=1e-5)


@pytest.mark.parametrize("N", [500, 130, 97])
def test_wide_mmd_eval_symmetric_matches_full(N):
    """The matrix-core MMD's evaluation (loss only: pred-pred tiles left of each row
    block's diagonal skipped, those right of it counted twice, blocks rotated over the
    XCDs per model) sums to the loss the training launch computes over every tile; the
    true-true launch (also symmetric) against the fp64 oracle's constant term."""
    from cgnn_amd import native
    from cgnn_amd.engine.batch import mmd_mfma_geometry, padded_dim
    hip = native.hip()
    d, R = 200, 3
    D = padded_dim(d)
    g = torch.Generator().manual_seed(N)
    P = torch.zeros(R, D, N)
    T = torch.zeros(R, D, N)
    P[:, :d] = torch.randn(R, d, N, generator=g) * 0.3
    T[:, :d] = torch.randn(R, d, N, generator=g) * 0.3 + 0.05
    P, T = P.cuda(), T.cuda()
    pn, tn = (P * P).sum(1).contiguous(), (T * T).sum(1).contiguous()
    rb, chunks, tpc = mmd_mfma_geometry(N, R)
    st = torch.cuda.current_stream().cuda_stream
    gradp = torch.empty(chunks, R, D, N, device="cuda")
    full = torch.zeros(R, rb * chunks, device="cuda")
    ev = torch.zeros(R, rb * chunks, device="cuda")
    tt = torch.zeros(R, rb * chunks, device="cuda")
    hip.mmd_mfma(0, D, P.data_ptr(), T.data_ptr(), pn.data_ptr(), tn.data_ptr(), gradp.data_ptr(),
                 full.data_ptr(), N, R, chunks, tpc, 1.0, st)
    hip.mmd_mfma(1, D, P.data_ptr(), T.data_ptr(), pn.data_ptr(), tn.data_ptr(), gradp.data_ptr(),
                 ev.data_ptr(), N, R, chunks, tpc, 0.0, st)
    hip.mmd_mfma(2, D, T.data_ptr(), T.data_ptr(), tn.data_ptr(), tn.data_ptr(), gradp.data_ptr(),
                 tt.data_ptr(), N, R, chunks, tpc, 0.0, st)
    np.testing.assert_allclose(ev.sum(1).cpu().numpy(), full.sum(1).cpu().numpy(), rtol=2e-5)
    # the true-true sum of the seven-bandwidth kernel, fp64
    Td = T[:, :d].double().cpu()
    d2 = ((Td[:, :, :, None] - Td[:, :, None, :]) ** 2).sum(1)
    from cgnn_amd.engine.reference import GAMMAS
    ref = sum(torch.exp(-gm * d2) for gm in GAMMAS).sum((1, 2))
    np.testing.assert_allclose(tt.sum(1).cpu().numpy(), ref.numpy(), rtol=1e-4)
