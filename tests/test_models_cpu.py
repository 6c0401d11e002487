"""End-to-end model / search behaviour on the CPU oracle path (tiny epochs)."""
import os

import numpy as np
import pandas as pd
import pytest

import cgnn
from cgnn_amd.engine.evaluator import GraphEvaluator
from cgnn_amd.search.hill_climbing import exploratory_hill_climbing, hill_climbing, tabu_search
from cgnn_amd.search.confounders import hill_climbing_confounders
from cgnn_amd.utils.graph import DirectedGraph, UndirectedGraph
from cgnn_amd.utils.metrics import METRICS, aupr, orientation_scores, shd, sign_accuracy
from cgnn_amd.utils.settings import SETTINGS

from conftest import example, have_example

TINY = dict(nb_runs=2, train_epochs=15, test_epochs=4, h_layer_dim=10, gpu=False)


@pytest.fixture(autouse=True)
def _cpu_settings(monkeypatch):
    monkeypatch.setattr(SETTINGS, "GPU", False)
    yield


def chain_data(n=120, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.normal(size=n)
    b = np.tanh(1.5 * a) + 0.3 * rng.normal(size=n)
    c = b ** 2 + 0.3 * rng.normal(size=n)
    return pd.DataFrame({"A": a, "B": b, "C": c})


def test_gnn_predict_proba_range_and_batch_equivalence():
    df = chain_data()
    m = cgnn.GNN(backend="TensorFlow")
    p1 = m.predict_proba(df.A.values, df.B.values, 0, **TINY)
    p2 = m.predict_proba_batch([(df.A.values, df.B.values, 0), (df.B.values, df.C.values, 1)], **TINY)
    assert -1 < p1 < 1
    assert abs(p2[0] - p1) < 1e-12          # batching does not change a pair's result
    assert len(m.last_run_scores) == 2 and len(m.last_run_scores[0][0]) == TINY["nb_runs"]


def test_predict_dataset_and_printout(tmp_path):
    from cgnn_amd.utils.formats import write_cepc_pairs, CCEPC_PairsFileReader
    df = chain_data(80)
    f = tmp_path / "pairs.csv"
    write_cepc_pairs(f, ["p0", "p1"], [df.A, df.B], [df.B, df.C])
    data = CCEPC_PairsFileReader(f)
    out = tmp_path / "printout.csv"
    preds = cgnn.GNN().predict_dataset(data, printout=str(out), **TINY)
    log = pd.read_csv(out)
    assert list(log.columns) == ["SampleID", "Predictions"]
    assert list(log.SampleID) == ["p0", "p1"]
    np.testing.assert_allclose(log.Predictions.values, preds)


def test_orient_graph_gives_dag_with_weights():
    df = chain_data()
    umg = UndirectedGraph()
    umg.add("A", "B")
    umg.add("B", "C")
    umg.add("A", "C")
    dag = cgnn.GNN().orient_graph(df, umg, **TINY)
    assert not dag.is_cyclic()
    assert len(dag.get_list_edges()) == 3
    assert all(0 <= w <= 1 for _, _, w in dag.get_list_edges())


def test_orient_graph_confounders_keeps_skeleton():
    df = chain_data()
    umg = UndirectedGraph()
    umg.add("A", "B")
    umg.add("B", "C")
    dag = cgnn.GNN().orient_graph_confounders(df, umg, **TINY)
    assert dag.skeleton is umg and not dag.is_cyclic()


def _toy_dag():
    g = DirectedGraph()
    g.add("B", "A", 0.1)
    g.add("B", "C", 0.2)
    return g


def test_cgnn_hill_climbing_runs_and_is_acyclic():
    df = chain_data()
    out = cgnn.CGNN(backend="TensorFlow").orient_directed_graph(df, _toy_dag(), **TINY)
    assert not out.is_cyclic()
    assert len(out.get_list_edges()) == 2
    assert np.isfinite(out.search_score)


def test_hill_climbing_speculation_width_does_not_change_result():
    df = chain_data()
    r1 = hill_climbing(_toy_dag(), df, None, speculation=1, **TINY)
    r8 = hill_climbing(_toy_dag(), df, None, speculation=8, **TINY)
    assert r1.canonical_key() == r8.canonical_key()
    assert r1.search_score == r8.search_score


def test_hill_climbing_checkpoint_resume(tmp_path):
    df = chain_data()
    ck = str(tmp_path / "hc.json")
    full = hill_climbing(_toy_dag(), df, None, **TINY)
    first = hill_climbing(_toy_dag(), df, None, checkpoint=ck, **TINY)
    assert os.path.exists(ck)
    resumed = hill_climbing(_toy_dag(), df, None, checkpoint=ck, **TINY)
    assert first.canonical_key() == full.canonical_key() == resumed.canonical_key()


def test_legacy_plugin_run_function():
    df = chain_data()
    calls = []

    def fake_run(data, graph, idx, run, **kw):
        calls.append((idx, run))
        # prefer A -> B
        return 1.0 if graph.has_edge("B", "A") else 0.5

    out = hill_climbing(_toy_dag(), df, fake_run, nb_runs=3, gpu=False)
    assert out.has_edge("A", "B")
    assert len(calls) % 3 == 0 and calls


def test_exploratory_hill_climbing_and_tabu():
    df = chain_data()
    e = exploratory_hill_climbing(_toy_dag(), df, None, nb_loops=3, **TINY)
    assert not e.is_cyclic()
    t = tabu_search(_toy_dag(), df, None, max_iter=2, patience=1, **TINY)
    assert not t.is_cyclic() and np.isfinite(t.search_score)


def test_cgnn_confounders_hill_climbing():
    df = chain_data()
    skel = UndirectedGraph()
    skel.add("A", "B")
    skel.add("B", "C")
    skel.add("A", "C")
    dag = DirectedGraph(skeleton=skel)
    dag.add("A", "B", 0.3)
    dag.add("B", "C", 0.2)
    out = cgnn.CGNN_confounders().orient_directed_graph(df, dag, **TINY)
    assert not out.is_cyclic()
    assert set(map(tuple, out.get_list_edges(return_weights=False))) <= {
        ("A", "B"), ("B", "A"), ("B", "C"), ("C", "B"), ("A", "C"), ("C", "A")}
    assert hasattr(out, "confounders")


def test_orient_undirected_graph_end_to_end():
    df = chain_data()
    umg = UndirectedGraph()
    umg.add("A", "B")
    umg.add("B", "C")
    out = cgnn.CGNN().predict(df, umg, **TINY)
    assert isinstance(out, DirectedGraph) and not out.is_cyclic()


def test_create_graph_from_data_raises():
    with pytest.raises(ValueError):
        cgnn.CGNN().predict(chain_data(), None)


def test_evaluator_penalty_and_nan_filter(monkeypatch):
    df = chain_data()
    cfg = SETTINGS.snapshot(**TINY)
    skel = UndirectedGraph()
    skel.add("A", "B")
    g = DirectedGraph(skeleton=skel)
    g.add("A", "B")
    ev = GraphEvaluator(df[["A", "B"]], cfg, mode="confounders", nodes=["A", "B"])
    raw = ev.run_scores([g])
    s = ev([g])[0]
    assert abs(s - (raw.mean() + cfg.complexity_graph_param)) < 1e-9
    monkeypatch.setenv("CGNN_FAULT", "nan@job:0")
    s2 = ev([g])[0]
    assert abs(s2 - raw[0, 1] - cfg.complexity_graph_param) < 1e-9   # run 0 dropped
    assert METRICS.last("dropped_runs")["count"] == 1


def test_cgnn_model_object_api():
    from cgnn.CGNN import CGNN_tf, run_CGNN_tf
    df = chain_data()
    g = DirectedGraph()
    g.add("A", "B")
    m = CGNN_tf(len(df), g, 0, 0, **TINY)
    m.train(df[["A", "B"]].values)
    score = m.evaluate(df[["A", "B"]].values)
    gen = m.generate(df[["A", "B"]].values)
    assert np.isfinite(score) and gen.shape == (len(df), 2)
    assert np.isfinite(run_CGNN_tf(df, g, 0, 0, **TINY))


def test_cgnn_model_verbose_prints_every_100_iterations(capsys):
    """CGNN_model.train / evaluate(verbose=True) print the reference's progress line
    (CGNN.py:123-127, 147-149) at iterations 0, 100, 200, ...; the score is the same as
    a silent run's (same draws)."""
    from cgnn.CGNN import CGNN_tf
    df = chain_data(n=60)
    g = DirectedGraph()
    g.add("A", "B")
    g.add("B", "C")
    kw = dict(TINY, train_epochs=205, test_epochs=150)
    data = df[["A", "B", "C"]].values
    m = CGNN_tf(len(df), g, 0, 3, **kw)
    m.train(data, verbose=True)
    score = m.evaluate(data, verbose=True)
    lines = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Pair:")]
    its = [int(l.split("Iter:")[1].split(",")[0]) for l in lines]
    assert its == [0, 100, 200, 0, 100]
    assert all(l.startswith("Pair:3, Run:0, Iter:") for l in lines)
    hist = m._trainer.loss_history[0]
    assert float(lines[1].split("score:")[1]) == pytest.approx(hist[100], rel=1e-6)
    q = CGNN_tf(len(df), g, 0, 3, **kw)
    q.train(data, verbose=False)
    s2 = q.evaluate(data, verbose=False)
    assert capsys.readouterr().out.count("Pair:") == 0
    assert s2 == pytest.approx(score, rel=1e-9)


def test_gnn_plugin_names():
    from cgnn.GNN import GNN_tf, tf_run_instance
    df = chain_data()
    m = np.stack([df.A.values, df.B.values], 1)
    xy, yx = tf_run_instance(m, 0, 0, **TINY)
    assert np.isfinite(xy) and np.isfinite(yx)
    g = GNN_tf(len(m), 0, 0, **TINY)
    g.train(m)
    assert np.isfinite(g.evaluate(m))


def test_metrics():
    t = DirectedGraph()
    t.add("a", "b")
    t.add("b", "c")
    p = DirectedGraph()
    p.add("b", "a")
    p.add("b", "c")
    p.add("a", "c")
    assert shd(p, t) == 2 and shd(p, t, double_for_anticausal=True) == 3
    assert orientation_scores(p, t)["tp"] == 1
    assert sign_accuracy([0.3, -0.2, 0.1], [1, 1, 1]) == pytest.approx(2 / 3)
    assert aupr([("a", "b", 0.9), ("x", "y", 0.5), ("b", "c", 0.1)], t) == pytest.approx((1 + 2 / 3) / 2)


@pytest.mark.skipif(not have_example("Example_graph_skeleton.csv"), reason="reference examples absent")
def test_reference_example_files_load():
    umg = UndirectedGraph(pd.read_csv(example("Example_graph_skeleton.csv")))
    assert len(umg.get_list_edges_without_duplicate()) == 30
    target = DirectedGraph(pd.read_csv(example("Example_graph_target.csv")))
    assert not target.is_cyclic()
    data = pd.read_csv(example("Example_graph_numdata.csv"))
    assert data.shape == (500, 22)


def test_compat_scores_pairwise_mean_and_candidate_keys():
    """SETTINGS.compat_scores: (1) the pairwise score averages every run, a non-finite
    one propagating (GNN.py:196-197) -- the default drops it; (2) HC candidates draw
    runs of their own (keys / subsamples keyed by the edge set), while the default
    shares run r's key across candidates (common random numbers)."""
    import numpy as np
    import pandas as pd
    from cgnn_amd.engine.evaluator import GraphEvaluator
    from cgnn_amd.models.gnn import pair_score
    from cgnn_amd.utils.graph import DirectedGraph
    from cgnn_amd.utils.settings import SETTINGS
    s = np.array([1.0, 2.0, np.nan, 2.5, 1.0, 2.0])
    ab, ba, p = pair_score(s)
    assert ab == 1.0 and ba == pytest.approx(13 / 6) and np.isfinite(p)
    ab, ba, p = pair_score(s, compat=True)
    assert np.isnan(ab) and np.isnan(p)
    rng = np.random.default_rng(0)
    df = pd.DataFrame(rng.standard_normal((40, 3)), columns=["A", "B", "C"])
    g1, g2 = DirectedGraph(), DirectedGraph()
    g1.add("A", "B")
    g1.add("B", "C")
    g2.add("B", "A")
    g2.add("B", "C")
    nodes = ["A", "B", "C"]
    ev = GraphEvaluator(df, SETTINGS.snapshot(nb_runs=3, gpu=False), nodes=nodes)
    assert [k for _, k in ev._runs(g1)] == [k for _, k in ev._runs(g2)]
    evc = GraphEvaluator(df, SETTINGS.snapshot(nb_runs=3, gpu=False, compat_scores=True), nodes=nodes)
    k1, k2 = [k for _, k in evc._runs(g1)], [k for _, k in evc._runs(g2)]
    assert len(set(k1 + k2)) == 6                     # every (candidate, run) its own stream
    assert k1 == [k for _, k in evc._runs(g1.copy())]  # a pure function of the edge set
    tiny = dict(train_epochs=3, test_epochs=2, h_layer_dim=5)
    evc = GraphEvaluator(df, SETTINGS.snapshot(nb_runs=2, gpu=False, compat_scores=True, **tiny), nodes=nodes)
    a = evc.run_scores([g1, g2])
    b = evc.run_scores([g2, g1])                      # batch position does not matter
    np.testing.assert_array_equal(a, b[::-1])
    assert not np.array_equal(a[0], a[1])


def _plugin(data, graph, idx, run, **kwargs):
    """A deterministic, picklable run_cgnn_function plug-in."""
    return float(idx) * 10.0 + run + 0.5 * len(graph.get_list_edges())


def test_plugin_nb_jobs_matches_sequential():
    """User run_cgnn_function plug-ins go through a joblib pool with nb_jobs > 1 (the
    reference's Parallel(n_jobs=NB_JOBS)); the scores equal the one-process loop."""
    import numpy as np
    import pandas as pd
    from cgnn_amd.engine.evaluator import GraphEvaluator
    from cgnn_amd.utils.graph import DirectedGraph
    from cgnn_amd.utils.settings import SETTINGS
    df = pd.DataFrame(np.zeros((5, 2)), columns=["A", "B"])
    g = DirectedGraph()
    g.add("A", "B")
    h = DirectedGraph()
    h.add("B", "A")
    out = []
    for jobs in (1, 4):
        ev = GraphEvaluator(df, SETTINGS.snapshot(nb_runs=3, nb_jobs=jobs, gpu=False), nodes=["A", "B"],
                            legacy_fn=_plugin)
        out.append(ev.run_scores([g, h, g]))
    np.testing.assert_array_equal(out[0], out[1])
    assert out[0][2, 1] == 21.5
