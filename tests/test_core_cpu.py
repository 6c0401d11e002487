"""Settings, formats, Philox RNG, DAG programs and the fp64 oracle (CPU)."""
import math
import os

import numpy as np
import pandas as pd
import pytest
import torch

import cgnn
from cgnn_amd.engine.program import (PROG_HDR, NODE_REC, program_for_confounders, program_for_dag,
                                     program_for_pair, pack_programs)
from cgnn_amd.engine.reference import (GAMMAS, ReferenceTrainer, mmd_loss_dense, rff_frequencies,
                                       rff_mmd_loss)
from cgnn_amd.utils import philox
from cgnn_amd.utils.formats import CCEPC_PairsFileReader, standardize, write_cepc_pairs
from cgnn_amd.utils.graph import DirectedGraph, UndirectedGraph
from cgnn_amd.utils.settings import DefaultSettings

from conftest import example, have_example


# ------------------------------------------------------------------ settings
def test_settings_defaults_and_slots():
    s = DefaultSettings()
    assert (s.NB_RUNS, s.NB_JOBS, s.GPU, s.NB_GPU, s.GPU_OFFSET) == (32, 1, True, 1, 0)
    assert (s.learning_rate, s.init_weights, s.max_nb_points) == (0.01, 0.05, 1500)
    assert (s.h_layer_dim, s.train_epochs, s.test_epochs) == (20, 1000, 500)
    assert (s.use_Fast_MMD, s.nb_vectors_approx_MMD, s.complexity_graph_param) == (False, 100, 5e-5)
    with pytest.raises(AttributeError):
        s.nb_runs = 3      # typo'd attribute (lower case) must raise, as with __slots__


def test_snapshot_kwargs_precedence():
    s = DefaultSettings()
    s.NB_RUNS = 8
    c = s.snapshot(init_std=0.1, nb_runs=4, h_layer_dim=30)
    assert c.init_std == 0.1 and c.nb_runs == 4 and c.h_layer_dim == 30
    assert s.snapshot().nb_runs == 8


def test_env_override(monkeypatch):
    monkeypatch.setenv("CGNN_NB_RUNS", "5")
    monkeypatch.setenv("CGNN_USE_FAST_MMD", "1")
    s = DefaultSettings()
    assert s.NB_RUNS == 5 and s.use_Fast_MMD is True


# ------------------------------------------------------------------ formats
def test_standardize_matches_population_scale():
    x = np.random.default_rng(0).normal(3, 2, size=(100, 3))
    z = standardize(x)
    np.testing.assert_allclose(z.mean(0), 0, atol=1e-12)
    np.testing.assert_allclose(z.std(0), 1, atol=1e-12)
    assert np.all(standardize(np.ones(5)) == 0)


def test_cepc_roundtrip(tmp_path):
    a = [np.arange(5.0), np.array([1.5, -2.0, 3.0])]
    b = [np.arange(5.0) ** 2, np.array([0.0, 1.0, 2.0])]
    p = tmp_path / "pairs.csv"
    write_cepc_pairs(p, ["p1", "p2"], a, b)
    df = CCEPC_PairsFileReader(p, scale=False)
    assert list(df.SampleID) == ["p1", "p2"]
    np.testing.assert_allclose(df.A[1], a[1])
    np.testing.assert_allclose(df.B[0], b[0])
    dfs = CCEPC_PairsFileReader(p, scale=True)
    np.testing.assert_allclose(dfs.A[0], standardize(a[0]))


@pytest.mark.skipif(not have_example("Example_pairwise_pairs.csv"), reason="reference examples absent")
def test_reads_reference_pairs_file():
    df = CCEPC_PairsFileReader(example("Example_pairwise_pairs.csv"))
    assert len(df) == 5 and all(len(a) == 1500 for a in df.A)


# ------------------------------------------------------------------ philox
def test_philox_known_answer():
    # Random123 known-answer vectors for philox4x32-10
    out = philox.philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(x) for x in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    out = philox.philox4x32_10(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF)
    assert [int(x) for x in out] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_philox_normals_are_standard():
    z = philox.normal(1, 2, np.arange(200000, dtype=np.uint32), 3, 4, philox.RNG_NODE_NOISE)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    z2 = philox.normal(1, 2, np.arange(10, dtype=np.uint32), 3, 5, philox.RNG_NODE_NOISE)
    assert not np.allclose(z[:10], z2)          # a different step draws fresh noise


def test_model_keys_are_stable():
    assert philox.model_key(0, "a", 1) == philox.model_key(0, "a", 1)
    assert philox.model_key(0, "a", 1) != philox.model_key(0, "a", 2)


# ------------------------------------------------------------------ programs
def test_program_layout_and_param_count():
    g = DirectedGraph()
    for a, b in [("x", "y"), ("x", "z"), ("y", "z")]:
        g.add(a, b)
    H = 20
    p = program_for_dag(g, H)
    recs = list(p.node_records())
    assert [r[0] for r in recs] == [0, 1, 2]          # generation order x, y, z
    assert [len(r[2]) for r in recs] == [0, 1, 2]     # parent counts
    assert p.n_params == sum((len(r[2]) + 1 + 2) * H + 1 for r in recs)
    assert p.max_in == 3


def test_confounder_program_shares_edge_noise():
    skel = UndirectedGraph()
    skel.add("a", "b")
    skel.add("b", "c")
    g = DirectedGraph(skeleton=skel)
    g.add("a", "b")
    p = program_for_confounders(g, 5)
    recs = {r[0]: r for r in p.node_records()}
    # every node gets one confounder input per skeleton neighbour; b sees both edges
    assert sorted(recs[1][3]) == [0, 1]
    assert recs[0][3] == [0] and recs[2][3] == [1]
    assert p.n_conf == 2


def test_pair_program_clamps_cause():
    p = program_for_pair(30)
    recs = list(p.node_records())
    assert recs[0][1] == 1 and recs[1][1] == 0 and recs[1][2] == [0]
    assert p.n_params == (2 + 2) * 30 + 1


def _check_schedule(prog):
    from cgnn_amd.engine.program import stage_schedule
    sched, wf, wb = stage_schedule(prog)
    nf, nb, fb, bb = (int(x) for x in sched[:4])
    recs = list(prog.node_records())
    var_of = [r[0] for r in recs]
    def stages(base, n):
        starts = sched[base:base + n + 1]
        items = sched[base + n + 1:]
        return [[int(k) for k in items[starts[i]:starts[i + 1]]] for i in range(n)]
    fwd, bwd = stages(fb, nf), stages(bb, nb)
    # forward: every record once; parents strictly earlier
    assert sorted(k for st in fwd for k in st) == list(range(len(recs)))
    stage_of_var = {var_of[k]: i for i, st in enumerate(fwd) for k in st}
    for k, (var, kind, pars, confs, poff, nin) in enumerate(recs):
        for p in pars:
            assert stage_of_var[p] < stage_of_var[var]
    # backward: every generated record once; children before parents; no sub-stage
    # shares a parent
    gen = sorted(k for k, r in enumerate(recs) if r[1] == 0)
    assert sorted(k for st in bwd for k in st) == gen
    pos = {var_of[k]: i for i, st in enumerate(bwd) for k in st}
    for st in bwd:
        seen = set()
        for k in st:
            pars = recs[k][2]
            assert not (seen & set(pars))
            seen |= set(pars)
            for p in pars:
                if p in pos:
                    assert pos[p] > pos[var_of[k]]
    assert wf == max(len(s) for s in fwd) and wb == max(len(s) for s in bwd)
    return fwd, bwd


def test_stage_schedule_levels_and_conflict_free_backward():
    """Level schedule of the wide-graph generator kernels (runtime dag_schedule)."""
    rng = np.random.default_rng(0)
    g = DirectedGraph()
    names = ["V%d" % k for k in range(60)]
    for k in range(1, 60):
        for p in rng.choice(k, size=min(k, int(rng.integers(1, 5))), replace=False):
            g.add(names[int(p)], names[k])
    fwd, bwd = _check_schedule(program_for_dag(g, 20))
    assert len(fwd) < 60 and len(bwd) >= len(fwd)
    # diamond: B and C share parent A -> separate backward sub-stages
    d = DirectedGraph()
    for a, b in [("A", "B"), ("A", "C"), ("B", "D"), ("C", "D")]:
        d.add(a, b)
    fwd, bwd = _check_schedule(program_for_dag(d, 5))
    assert [len(s) for s in fwd] == [1, 2, 1] and [len(s) for s in bwd] == [1, 1, 1, 1]
    _check_schedule(program_for_pair(7))
    skel = UndirectedGraph()
    skel.add("a", "b")
    skel.add("b", "c")
    c = DirectedGraph(skeleton=skel)
    c.add("a", "b")
    _check_schedule(program_for_confounders(c, 5))


def test_cyclic_graph_program_rejected():
    g = DirectedGraph()
    g.add("a", "b")
    g.add("b", "a")
    with pytest.raises(Exception):
        program_for_dag(g, 5)


# ------------------------------------------------------------------ oracle
def test_mmd_dense_matches_brute_force():
    rng = np.random.default_rng(1)
    p, t = rng.normal(size=(7, 3)), rng.normal(size=(7, 3))
    brute = 0.0
    X = np.vstack([p, t])
    s = np.r_[np.full(7, 1 / 7), np.full(7, -1 / 7)]
    for i in range(14):
        for j in range(14):
            d2 = ((X[i] - X[j]) ** 2).sum()
            brute += s[i] * s[j] * sum(math.exp(-g * d2) for g in GAMMAS)
    got = float(mmd_loss_dense(torch.tensor(p), torch.tensor(t)))
    assert abs(got - brute) < 1e-12


def test_mmd_analytic_gradient_matches_finite_difference():
    rng = np.random.default_rng(2)
    p = torch.tensor(rng.normal(size=(9, 2)), requires_grad=True)
    t = torch.tensor(rng.normal(size=(9, 2)))
    L = mmd_loss_dense(p, t)
    (g,) = torch.autograd.grad(L, p)
    # the fused kernel's closed form: g_i = 4/N^2 sum_j sign_j w_ij (x_j - p_i)
    N = 9
    X = torch.cat([p.detach(), t])
    sign = torch.cat([torch.ones(N), -torch.ones(N)]).double()
    d2 = torch.cdist(p.detach(), X) ** 2
    w = sum(gm * torch.exp(-gm * d2) for gm in GAMMAS)
    closed = 4.0 / N ** 2 * ((sign[None, :] * w)[:, :, None] * (X[None, :, :] - p.detach()[:, None, :])).sum(1)
    np.testing.assert_allclose(g.numpy(), closed.numpy(), rtol=1e-10, atol=1e-12)


def test_rff_frequencies_shape_and_scale():
    W = rff_frequencies((3, 4), 0, k=50, d=2)
    assert W.shape == (3, 350)
    assert torch.all((W[2] >= 0) & (W[2] <= 2 * math.pi))
    # block b has std 2*gamma_b (reference scaling, B12)
    assert abs(W[:2, 300:].std().item() / 100.0 - 1) < 0.25


def test_reference_trainer_decreases_loss():
    p = program_for_pair(20)
    rng = np.random.default_rng(0)
    x = rng.normal(size=300)
    y = np.tanh(2 * x) + 0.1 * rng.normal(size=300)
    data = standardize(np.stack([x, y], 0).T).T.astype(np.float32)
    tr = ReferenceTrainer([p], [data], [(1, 2)], 20, learning_rate=0.01)
    tr.train(60)
    h = tr.loss_history[0]
    assert np.mean(h[-10:]) < 0.7 * np.mean(h[:5])


def test_package_surface():
    """the reference's public names are importable from ``cgnn``."""
    assert set(cgnn.__all__) == {"DirectedGraph", "UndirectedGraph", "CGNN", "CGNN_confounders", "GNN"}
    for name in ("NB_RUNS", "NB_JOBS", "GPU", "NB_GPU", "GPU_OFFSET", "learning_rate", "init_weights",
                 "max_nb_points", "h_layer_dim", "train_epochs", "test_epochs", "use_Fast_MMD",
                 "nb_vectors_approx_MMD", "complexity_graph_param"):
        assert hasattr(cgnn.SETTINGS, name)
    assert callable(cgnn.utils.CCEPC_PairsFileReader)
    for name in ("MMD_loss_tf", "Fourier_MMD_Loss_tf", "MomentMatchingLoss_tf", "rp", "f1", "bandwiths_gamma"):
        assert hasattr(cgnn.utils.Loss, name)
    assert cgnn.generators.RandomGraphGenerator is not None
    from cgnn import CGNN as C, CGNN_confounders as CC, GNN as G  # noqa: F401
    from cgnn.CGNN import (CGNN_tf, run_CGNN_tf, hill_climbing, exploratory_hill_climbing,  # noqa: F401
                           tabu_search)
    from cgnn.CGNN_confounders import (CGNN_confounders_tf, run_CGNN_confounders_tf,  # noqa: F401
                                       hill_climbing_confounders)
    from cgnn.GNN import GNN_tf, tf_run_instance  # noqa: F401
    with pytest.raises(ValueError):
        cgnn.CGNN().create_graph_from_data(pd.DataFrame({"a": [1.0]}))


def test_moment_matching_loss_b8():
    from cgnn_amd.utils.loss import MomentMatchingLoss
    x = torch.randn(200, 2, dtype=torch.float64)
    assert float(MomentMatchingLoss(x, x, 3)) == 0.0
    y = x + 0.5
    one = float(MomentMatchingLoss(x, y, 1))         # the reference's default returned 0 (off by one)
    assert one == pytest.approx(float(torch.sqrt(((x.mean(0) - y.mean(0)) ** 2).sum())), rel=1e-12)
    assert float(MomentMatchingLoss(x, y, 2)) > one


def _dag_with_max_in(d, k, seed):
    """A DAG over d variables whose node d-1 has k parents, every other node <= 2."""
    rng = np.random.default_rng(seed)
    g = DirectedGraph()
    names = ["V%d" % i for i in range(d)]
    for i in range(1, d - 1):
        for p in rng.choice(i, size=min(i, 2), replace=False):
            g.add(names[int(p)], names[i])
    for p in rng.choice(d - 1, size=k, replace=False):
        g.add(names[int(p)], names[d - 1])
    return g


def test_device_batches_keep_each_program_on_its_own_kernel_family():
    """the generator kernels (per-sample or level-scheduled) are chosen per
    program, never from batch-wide maxima, so a candidate's score cannot depend on its
    batch-mates.  The family follows the variable count (per-sample up to 24 variables,
    level-scheduled above, profiles/r05_family), whatever a program's widest node: at
    d = 24 and d = 140, programs with 3 and 19 inputs on one node share their width's
    family, every batch keeps one family, and its combined shape keeps it."""
    from cgnn_amd.engine.batch import kernel_family
    from cgnn_amd.engine.scorer import Job, _group_batches
    H, N = 20, 50
    for d, fam in ((24, 1), (140, 2)):
        progs = [program_for_dag(_dag_with_max_in(d, k, s), H) for s, k in enumerate([3, 19, 3, 19, 3, 3, 19])]
        fams = [kernel_family(d, H, p.max_in, len(p.prog)) for p in progs]
        assert set(fams) == {fam}, (d, fams)
        data = np.zeros((d, N), np.float32)
        jobs = [Job(p, data, (0, i)) for i, p in enumerate(progs)]
        batches = _group_batches(jobs, 16, H=H)
        assert sorted(i for b in batches for i in b) == list(range(len(jobs)))
        for b in batches:
            ps = [progs[i] for i in b]
            assert kernel_family(d, H, max(p.max_in for p in ps), max(len(p.prog) for p in ps)) == fam
        # without H (the CPU reference path) only the shape matters
        assert len(_group_batches(jobs, 16)) == 1


@pytest.mark.parametrize("fast", [False, True])
def test_device_kernels_cover_every_width_to_2048(fast):
    """no CPU fallback below realistic widths -- every d <= 2048 (exact or
    Fourier MMD) has device kernels, for sparse DAGs and for nodes with many inputs."""
    from cgnn_amd.engine.batch import device_supported
    for d in (2, 22, 65, 200, 257, 300, 512, 1000, 1025, 1500, 2048):
        for max_in in (2, 8, 64):
            prog_len = 4 + 8 * d + d * min(max_in, d)
            assert device_supported(d, 20, min(max_in, d + 1), prog_len, fast_mmd=fast), (d, max_in)
