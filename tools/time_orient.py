"""Time ``CGNN().orient_directed_graph`` on the reference generator's default graph
(RandomGraphGenerator(num_nodes=200), generators/random_graph_generator.py:26) at the
reference settings (32 runs, 1000 train + 500 eval steps, h_layer_dim 20; Settings.py).

A full hill-climbing search on 200 variables scores hundreds of candidates per pass, so
the run is time-boxed: the evaluator stops the search after ``--seconds`` and the tool
prints the candidate evaluations per second it sustained (the unit SURVEY §6 asks for),
the model-steps per second behind them, and the time one full HC pass over the graph's
edges would take at that rate.

    python tools/time_orient.py --seconds 240
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Budget(Exception):
    pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=200)
    ap.add_argument("--points", type=int, default=500)
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--runs", type=int, default=32)
    ap.add_argument("--train", type=int, default=1000)
    ap.add_argument("--test", type=int, default=500)
    ap.add_argument("--h", type=int, default=20)
    ap.add_argument("--batch-models", type=int, default=0,
                    help="models per device batch (runs x candidates; 0: the SETTINGS default)")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import cgnn
    from cgnn_amd.generators import RandomGraphGenerator
    from cgnn_amd.search import hill_climbing as hc
    from cgnn_amd.utils.settings import SETTINGS

    gen = RandomGraphGenerator(num_nodes=a.nodes, number_points=a.points, seed=a.seed)
    graph, data = gen.generate(gen_cat=False)[:2]
    n_vars, n_edges = len(graph.get_list_nodes()), len(graph.get_list_edges())
    kw = dict(nb_runs=a.runs, train_epochs=a.train, test_epochs=a.test, h_layer_dim=a.h, gpu=True)
    if a.batch_models:
        kw["batch_models"] = a.batch_models
    state = {"cand": 0, "batches": 0, "t0": None, "first": None}
    make = hc.make_evaluator

    def timed_make(*args, **kwargs):
        ev = make(*args, **kwargs)
        inner = ev.__call__

        class Timed:
            def __getattr__(self, name):
                return getattr(ev, name)

            def __call__(self, graphs):
                graphs = list(graphs)
                if state["t0"] is None:
                    state["t0"] = time.perf_counter()
                t = time.perf_counter()
                out = inner(graphs)
                if state["first"] is None:
                    state["first"] = time.perf_counter() - t     # initial score (includes warm-up)
                    state["t1"] = time.perf_counter()
                else:
                    state["cand"] += len(graphs)
                    state["batches"] += 1
                el = time.perf_counter() - state["t1"]
                print(json.dumps({"batch": state["batches"], "candidates": state["cand"],
                                  "seconds": round(el, 1), "batch_s": round(time.perf_counter() - t, 2)}),
                      flush=True)
                if time.perf_counter() - state["t0"] > a.seconds:
                    raise _Budget()
                return out
        return Timed()

    hc.make_evaluator = timed_make
    t_start = time.perf_counter()
    finished = True
    try:
        cgnn.CGNN(backend="TensorFlow").orient_directed_graph(data, graph, **kw)
    except _Budget:
        finished = False
    t_end = time.perf_counter()
    steps = a.train + a.test
    el = t_end - state.get("t1", t_end)
    rate = state["cand"] / el if el > 0 else 0.0
    print(json.dumps({
        "bench": "orient_directed_graph", "variables": n_vars, "edges": n_edges, "points": a.points,
        "runs": a.runs, "train_steps": a.train, "test_steps": a.test, "h_layer_dim": a.h,
        "batch_models": int(SETTINGS.snapshot(**kw).batch_models),
        "initial_score_s": round(state["first"] or 0.0, 2),
        "candidates_scored": state["cand"], "batches": state["batches"], "seconds": round(el, 1),
        "candidate_evals_per_s": round(rate, 3),
        "model_steps_per_s": round(rate * a.runs * steps, 1),
        "hc_pass_s_projected": round(n_edges / rate, 1) if rate else None,
        "search_finished": finished, "wall_s": round(t_end - t_start, 1)}))


if __name__ == "__main__":
    main()
