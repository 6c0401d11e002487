"""Orient a skeleton into a DAG: pairwise GNN orientation, then CGNN hill
climbing (reference: run_CGNN_graph.py).  Writes the reference CSVs and reports
wall time and SHD / precision against <data>_target.csv."""
import argparse
import json
import os
import time

import _common  # noqa: F401
import pandas as pd

import cgnn
from cgnn_amd.utils.metrics import METRICS, orientation_scores, shd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--skeleton", default=None)
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--alg", default="HC", choices=["HC", "EHC", "tabu"])
    ap.add_argument("--runs", type=int, default=None)
    ap.add_argument("--train", type=int, default=None)
    ap.add_argument("--test", type=int, default=None)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--fast-mmd", action="store_true", help="SETTINGS.use_Fast_MMD (random Fourier features)")
    a = ap.parse_args()
    datafile = _common.data_path("Example_graph_numdata.csv", a.data)
    skeletonfile = _common.data_path("Example_graph_skeleton.csv", a.skeleton)
    cgnn.SETTINGS.GPU = True
    cgnn.SETTINGS.NB_GPU = 2
    cgnn.SETTINGS.NB_JOBS = 8
    cgnn.SETTINGS.NB_RUNS = a.runs or 32
    if a.train:
        cgnn.SETTINGS.train_epochs = a.train
    if a.test:
        cgnn.SETTINGS.test_epochs = a.test
    cgnn.SETTINGS.use_Fast_MMD = bool(a.fast_mmd)
    base = os.path.join(a.out_dir, os.path.basename(datafile))
    print("Processing " + datafile + "...")
    t0 = time.perf_counter()
    umg = cgnn.UndirectedGraph(pd.read_csv(skeletonfile))
    data = pd.read_csv(datafile)
    GNN = cgnn.GNN(backend="TensorFlow")
    p_directed_graph = GNN.orient_graph(data, umg, printout=base + '_printout.csv')
    t1 = time.perf_counter()
    pd.DataFrame(p_directed_graph.get_list_edges(descending=True),
                 columns=['Cause', 'Effect', 'Score']).to_csv(base + "_pairwise_predictions.csv")
    CGNN = cgnn.CGNN(backend="TensorFlow")
    directed_graph = CGNN.orient_directed_graph(data, p_directed_graph, alg=a.alg,
                                                checkpoint=a.checkpoint)
    t2 = time.perf_counter()
    pd.DataFrame(directed_graph.get_list_edges(descending=True),
                 columns=['Cause', 'Effect', 'Score']).to_csv(base + "_predictions.csv")
    res = {"workload": "graph", "alg": a.alg, "fast_mmd": bool(a.fast_mmd), "seconds_pairwise": round(t1 - t0, 3),
           "seconds_search": round(t2 - t1, 3), "seconds_total": round(t2 - t0, 3),
           "candidates_evaluated": (METRICS.last("candidates") or {}).get("total")}
    tfile = datafile.replace("_numdata.csv", "_target.csv")
    if os.path.exists(tfile):
        target = cgnn.DirectedGraph(pd.read_csv(tfile))
        res["shd_pairwise"] = shd(p_directed_graph, target)
        res["shd_cgnn"] = shd(directed_graph, target)
        res["cgnn_orientation"] = orientation_scores(directed_graph, target)
    print('Processed ' + datafile)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
