"""Micro-benchmark of one CGNN device batch: R models of a random DAG over d
variables (the shape of one hill-climbing candidate batch of the reference's
graph example: d=22, 30 edges, N=500, h=20, 32 runs x 8 candidates = 256).

    python tools/bench_cgnn_batch.py --d 22 --edges 30 --R 256 --train 200 --test 100
Prints one JSON line with the time per train step / eval step."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def random_dag_program(d, n_edges, H, seed, confounders=0):
    from cgnn_amd.engine.program import compile_program
    rng = np.random.default_rng(seed)
    pairs = [(i, j) for i in range(d) for j in range(i + 1, d)]
    pick = rng.choice(len(pairs), size=min(n_edges, len(pairs)), replace=False)
    perm = rng.permutation(d)
    nodes = ["V%d" % k for k in range(d)]
    parents = {n: [] for n in nodes}
    for k in pick:
        i, j = pairs[k]
        parents[nodes[perm[j]]].append(nodes[perm[i]])
    conf = None
    if confounders:
        conf = {n: [] for n in nodes}
        for c in range(confounders):
            a, b = rng.choice(d, 2, replace=False)
            conf[nodes[a]].append(c)
            conf[nodes[b]].append(c)
    return compile_program(nodes, parents, H, confounders=conf, n_conf=confounders)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=22)
    ap.add_argument("--edges", type=int, default=30)
    ap.add_argument("--conf", type=int, default=0)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--R", type=int, default=256)
    ap.add_argument("--h", type=int, default=20)
    ap.add_argument("--train", type=int, default=200)
    ap.add_argument("--test", type=int, default=100)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph replay (for PMC collection)")
    ap.add_argument("--generator", choices=["auto", "staged"], default="auto",
                    help="generator kernels: the batch's kernel family, or the level-scheduled ones (A/B)")
    a = ap.parse_args()
    import torch
    from cgnn_amd.engine.batch import DeviceTrainer
    from cgnn_amd.utils.philox import model_key
    prog = random_dag_program(a.d, a.edges, a.h, 0, a.conf)
    data = np.random.default_rng(1).normal(size=(a.d, a.n)).astype(np.float32)
    tr = DeviceTrainer([prog] * a.R, [data] * a.R, [model_key(0, r) for r in range(a.R)], a.h, "cuda:0",
                       use_fast_mmd=a.fast, graph_chunk=0 if a.eager else 50, generator=a.generator)
    tr.run(10, 10)                                   # warm-up: graph capture, first launches
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.start()
    tr.train(a.train)
    tr._join()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tr.evaluate(a.test)
    tr._join()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"bench": "cgnn_batch", "d": a.d, "edges": a.edges, "conf": a.conf, "N": a.n, "R": a.R,
                      "generator": "staged" if tr.staged else "per-sample",
                      "H": a.h, "us_per_train_step": 1e6 * (t1 - t0) / a.train,
                      "us_per_eval_step": 1e6 * (t2 - t1) / a.test,
                      "model_steps_per_s": a.R * (a.train + a.test) / (t2 - t0)}))


if __name__ == "__main__":
    main()
