"""Pairwise cause-effect inference on a CEPC pairs file
(reference: run_GNN_pairwise_inference.py).  Writes <data>_printout.csv and
<data>_predictions_GNN.csv in the reference formats, and reports wall time and
the sign accuracy against <data>_targets.csv when present."""
import argparse
import json
import os
import time

import _common  # noqa: F401
import numpy as np
import pandas as pd

import cgnn
from cgnn.utils import CCEPC_PairsFileReader as CC


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--fast-mmd", action="store_true", help="CGNN-Fourier setting (NB_RUNS=64)")
    ap.add_argument("--runs", type=int, default=None)
    ap.add_argument("--train", type=int, default=None)
    ap.add_argument("--test", type=int, default=None)
    a = ap.parse_args()
    datafile = _common.data_path("Example_pairwise_pairs.csv", a.data)
    cgnn.SETTINGS.GPU = True
    cgnn.SETTINGS.NB_GPU = 2
    cgnn.SETTINGS.NB_JOBS = 8
    cgnn.SETTINGS.h_layer_dim = 30
    cgnn.SETTINGS.use_Fast_MMD = a.fast_mmd
    cgnn.SETTINGS.NB_RUNS = 64 if a.fast_mmd else 32
    if a.runs:
        cgnn.SETTINGS.NB_RUNS = a.runs
    if a.train:
        cgnn.SETTINGS.train_epochs = a.train
    if a.test:
        cgnn.SETTINGS.test_epochs = a.test
    base = os.path.join(a.out_dir, os.path.basename(datafile))
    print("Processing " + datafile + "...")
    t0 = time.perf_counter()
    data = CC(datafile, scale=True)
    model = cgnn.GNN(backend="TensorFlow")
    predictions = model.predict_dataset(data, printout=base + '_printout.csv')
    dt = time.perf_counter() - t0
    pd.DataFrame(predictions, columns=["Predictions"]).to_csv(base + "_predictions_GNN.csv")
    res = {"workload": "pairwise", "pairs": len(data), "seconds": round(dt, 3),
           "runs": cgnn.SETTINGS.NB_RUNS, "fast_mmd": a.fast_mmd}
    tfile = datafile.replace("_pairs.csv", "_targets.csv")
    if os.path.exists(tfile):
        t = pd.read_csv(tfile)["Target"].values
        res["sign_accuracy"] = float(np.mean((np.array(predictions) > 0) == (t > 0)))
    print('Processed ' + datafile)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
