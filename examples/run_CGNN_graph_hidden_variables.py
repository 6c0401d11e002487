"""Orient a skeleton in the presence of hidden confounders
(reference: run_CGNN_graph_hidden_variables.py)."""
import argparse
import json
import os
import time

import _common  # noqa: F401
import pandas as pd

import cgnn
from cgnn_amd.utils.formats import standardize
from cgnn_amd.utils.metrics import METRICS, orientation_scores, shd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--skeleton", default=None)
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--runs", type=int, default=None)
    ap.add_argument("--train", type=int, default=None)
    ap.add_argument("--test", type=int, default=None)
    a = ap.parse_args()
    datafile = _common.data_path("Example_graph_confounders_numdata.csv", a.data)
    skeletonfile = _common.data_path("Example_graph_confounders_skeleton.csv", a.skeleton)
    cgnn.SETTINGS.GPU = True
    cgnn.SETTINGS.NB_GPU = 2
    cgnn.SETTINGS.NB_JOBS = 8
    cgnn.SETTINGS.NB_RUNS = a.runs or 32
    if a.train:
        cgnn.SETTINGS.train_epochs = a.train
    if a.test:
        cgnn.SETTINGS.test_epochs = a.test
    base = os.path.join(a.out_dir, os.path.basename(datafile))
    t0 = time.perf_counter()
    data = pd.read_csv(datafile)
    skeleton = cgnn.UndirectedGraph(pd.read_csv(skeletonfile))
    data = pd.DataFrame(standardize(data.values), columns=data.columns)
    GNN = cgnn.GNN(backend="TensorFlow")
    p_directed_graph = GNN.orient_graph_confounders(data, skeleton, printout=base + '_printout.csv')
    t1 = time.perf_counter()
    pd.DataFrame(p_directed_graph.get_list_edges(descending=True),
                 columns=['Cause', 'Effect', 'Score']).to_csv(base + "_pairwise_predictions.csv")
    model = cgnn.CGNN_confounders(backend="TensorFlow")
    directed_graph = model.orient_directed_graph(data, p_directed_graph)
    t2 = time.perf_counter()
    pd.DataFrame(directed_graph.get_list_edges(descending=True),
                 columns=['Cause', 'Effect', 'Score']).to_csv(base + "_confounders_predictions.csv")
    res = {"workload": "confounders", "seconds_pairwise": round(t1 - t0, 3),
           "seconds_search": round(t2 - t1, 3), "seconds_total": round(t2 - t0, 3),
           "candidates_evaluated": (METRICS.last("candidates") or {}).get("total"),
           "possible_confounders": [list(map(str, c)) for c in getattr(directed_graph, "confounders", [])]}
    tfile = datafile.replace("_numdata.csv", "_target.csv")
    if os.path.exists(tfile):
        target = cgnn.DirectedGraph(pd.read_csv(tfile))
        res["shd_pairwise"] = shd(p_directed_graph, target)
        res["shd_cgnn"] = shd(directed_graph, target)
        res["cgnn_orientation"] = orientation_scores(directed_graph, target)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
