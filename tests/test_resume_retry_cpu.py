"""Failure handling and observability: resume of every structure
search from its checkpoint after a crash, retry of non-finite runs
(``max_retries`` under ``CGNN_FAULT`` injection) and ``CGNN_PROFILE`` phase timers."""
import hashlib
import os

import numpy as np
import pandas as pd
import pytest

import cgnn
from cgnn_amd.engine.evaluator import GraphEvaluator
from cgnn_amd.search.confounders import hill_climbing_confounders
from cgnn_amd.search.hill_climbing import exploratory_hill_climbing, hill_climbing, tabu_search
from cgnn_amd.utils.graph import DirectedGraph, UndirectedGraph
from cgnn_amd.utils.metrics import METRICS
from cgnn_amd.utils.settings import SETTINGS

TINY = dict(nb_runs=2, train_epochs=15, test_epochs=4, h_layer_dim=10, gpu=False)


@pytest.fixture(autouse=True)
def _cpu_settings(monkeypatch):
    monkeypatch.setattr(SETTINGS, "GPU", False)
    yield


def _data(cols, n=60, seed=0):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({c: rng.normal(size=n) for c in cols})


class Scorer:
    """Deterministic plug-in run function (score = hash of the edge set); raises
    after ``crash_after`` calls to simulate a killed job."""

    def __init__(self, crash_after=None):
        self.calls, self.crash_after = 0, crash_after

    def __call__(self, data, graph, idx, run, **kw):
        self.calls += 1
        if self.crash_after is not None and self.calls > self.crash_after:
            raise RuntimeError("simulated crash")
        key = repr(sorted(graph.get_list_edges(order_by_weight=False, return_weights=False)))
        h = hashlib.sha256((key + str(run)).encode()).digest()
        return int.from_bytes(h[:4], "little") / 2 ** 32


def _crash_then_resume(search, make_graph, data, tmp_path, crash_after, **kw):
    full = search(make_graph(), data, Scorer(), **kw)
    ck = str(tmp_path / "state.json")
    with pytest.raises(RuntimeError):
        search(make_graph(), data, Scorer(crash_after), checkpoint=ck, **kw)
    assert os.path.exists(ck)                  # the crash came after at least one saved state
    resumed_scorer = Scorer()
    resumed = search(make_graph(), data, resumed_scorer, checkpoint=ck, **kw)
    return full, resumed, resumed_scorer.calls


def _chain(names):
    g = DirectedGraph()
    for a, b in zip(names[:-1], names[1:]):
        g.add(a, b, 0.1)
    g.add(names[0], names[2], 0.2)
    return g


def test_confounder_hill_climbing_resumes_after_crash(tmp_path):
    names = ["A", "B", "C", "D", "E"]
    data = _data(names)

    def make():
        skel = UndirectedGraph()
        for a, b in [("A", "B"), ("B", "C"), ("C", "D"), ("D", "E"), ("A", "C"), ("B", "E")]:
            skel.add(a, b)
        g = DirectedGraph(skeleton=skel)
        for a, b in [("A", "B"), ("B", "C"), ("C", "D"), ("D", "E"), ("A", "C")]:
            g.add(a, b, 0.1)
        return g

    full, resumed, calls = _crash_then_resume(hill_climbing_confounders, make, data, tmp_path, 9, nb_runs=3,
                                              gpu=False, speculation=2)
    assert resumed.canonical_key() == full.canonical_key()
    assert resumed.search_score == full.search_score
    assert resumed.confounders == full.confounders
    assert 0 < calls   # resumed work only: the initial score is not recomputed


def test_ehc_resumes_after_crash(tmp_path):
    names = ["A", "B", "C", "D"]
    full, resumed, _ = _crash_then_resume(exploratory_hill_climbing, lambda: _chain(names), _data(names),
                                          tmp_path, 7, nb_loops=6, exploration_factor=2, nb_runs=2, gpu=False)
    assert resumed.canonical_key() == full.canonical_key() and resumed.search_score == full.search_score


def test_tabu_resumes_after_crash(tmp_path):
    names = ["A", "B", "C", "D"]
    full, resumed, _ = _crash_then_resume(tabu_search, lambda: _chain(names), _data(names), tmp_path, 9,
                                          max_iter=5, patience=3, nb_runs=2, gpu=False)
    assert resumed.canonical_key() == full.canonical_key() and resumed.search_score == full.search_score


def test_hill_climbing_resumes_after_crash(tmp_path):
    names = ["A", "B", "C", "D"]
    full, resumed, _ = _crash_then_resume(hill_climbing, lambda: _chain(names), _data(names), tmp_path, 5,
                                          nb_runs=2, gpu=False, speculation=1)
    assert resumed.canonical_key() == full.canonical_key() and resumed.search_score == full.search_score


def test_max_retries_recovers_injected_nan(monkeypatch):
    df = _data(["A", "B"])
    g = DirectedGraph()
    g.add("A", "B")
    monkeypatch.setenv("CGNN_FAULT", "nan@job:0")
    METRICS.clear()
    ev = GraphEvaluator(df, SETTINGS.snapshot(**TINY), nodes=["A", "B"])
    raw = ev.run_scores([g])
    assert np.isnan(raw[0, 0]) and METRICS.last("dropped_runs")["count"] == 1
    METRICS.clear()
    ev = GraphEvaluator(df, SETTINGS.snapshot(max_retries=2, **TINY), nodes=["A", "B"])
    raw = ev.run_scores([g])
    assert np.all(np.isfinite(raw))
    assert METRICS.last("retried_runs")["recovered"] == 1 and METRICS.last("dropped_runs") is None
    # the same through the settings singleton and a public entry point
    monkeypatch.setattr(SETTINGS, "max_retries", 1)
    METRICS.clear()
    p = cgnn.GNN().predict_proba(df["A"].values, df["B"].values, **TINY)
    assert np.isfinite(p) and METRICS.last("retried_runs")["count"] == 1


def test_profile_timers_record_phases(monkeypatch):
    monkeypatch.setenv("CGNN_PROFILE", "1")
    METRICS.clear()
    df = _data(["A", "B", "C"])
    g = DirectedGraph()
    g.add("A", "B", 0.1)
    g.add("B", "C", 0.2)
    cgnn.CGNN().orient_directed_graph(df, g, **TINY)
    names = {e["name"] for e in METRICS.events if e["event"] == "phase"}
    assert {"score_jobs", "search:HC", "search:initial_score", "search:candidates"} <= names
    assert all(e["seconds"] >= 0 for e in METRICS.events if e["event"] == "phase")
    monkeypatch.delenv("CGNN_PROFILE")
    METRICS.clear()
    cgnn.CGNN().orient_directed_graph(df, g, **TINY)
    assert not [e for e in METRICS.events if e["event"] == "phase"]


def test_confounder_hill_climbing_speculation_keeps_the_sequential_result():
    """Speculative windows (the candidates of several skeleton edges in one batch)
    accept exactly the sequential sequence of changes."""
    names = ["A", "B", "C", "D", "E", "F"]
    data = _data(names)

    def make():
        skel = UndirectedGraph()
        for a, b in [("A", "B"), ("B", "C"), ("C", "D"), ("D", "E"), ("A", "C"), ("B", "E"), ("E", "F"), ("A", "F")]:
            skel.add(a, b)
        g = DirectedGraph(skeleton=skel)
        for a, b in [("A", "B"), ("C", "B"), ("C", "D"), ("E", "D"), ("A", "C"), ("F", "E")]:
            g.add(a, b, 0.1)
        return g

    # the deterministic hash scorer accepts changes often: windows are cut frequently
    seq = hill_climbing_confounders(make(), data, Scorer(), nb_runs=3, gpu=False, speculation=2)
    for w in (4, 7, 64):
        spec = hill_climbing_confounders(make(), data, Scorer(), nb_runs=3, gpu=False, speculation=w)
        assert spec.canonical_key() == seq.canonical_key()
        assert spec.search_score == seq.search_score
        assert spec.confounders == seq.confounders


def test_fault_injection_keeps_job_ids_across_short_long_split(monkeypatch):
    """A call mixing long-N jobs (sample-sharded trainer) and short ones (batched
    engine) recurses on the short subset: CGNN_FAULT job numbers still address the
    caller's jobs, and max_retries recovers them (the recursion re-indexed)."""
    from cgnn_amd.engine.program import program_for_pair
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.philox import model_key
    rng = np.random.default_rng(0)

    def job(N, k):
        x = rng.standard_normal(N)
        y = np.tanh(x) + 0.3 * rng.standard_normal(N)
        return Job(program_for_pair(6), np.stack([x, y]).astype(np.float32), model_key(5, k))

    jobs = [job(300, 0), job(40, 1), job(300, 2), job(40, 3)]     # long, short, long, short
    cfg = SETTINGS.snapshot(train_epochs=3, test_epochs=2, h_layer_dim=6, gpu=False, long_n_min=100)
    clean = score_jobs(jobs, cfg, max_retries=0)
    assert np.all(np.isfinite(clean))
    for bad in (3, 2):                               # a short job, then a long one
        monkeypatch.setenv("CGNN_FAULT", "nan@job:%d" % bad)
        s = score_jobs(jobs, cfg, max_retries=0)
        assert np.isnan(s[bad]) and np.all(np.isfinite(np.delete(s, bad))), (bad, s)
        np.testing.assert_array_equal(np.delete(s, bad), np.delete(clean, bad))
        r = score_jobs(jobs, cfg, max_retries=1)
        assert np.all(np.isfinite(r)), (bad, r)
