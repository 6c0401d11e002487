"""Time the long-N CGNN path (engine/sharded.py): one pairwise / DAG job with N samples
(the reference caps N at 1500 by subsampling), train K + eval K/2 steps; on W ranks
(torchrun) the samples are split over the ranks.  Prints one JSON line (rank 0).

    python tools/bench_long_n.py --N 100000 --d 2 --train 20 --test 10
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=100000)
    ap.add_argument("--d", type=int, default=2)
    ap.add_argument("--h", type=int, default=20)
    ap.add_argument("--train", type=int, default=20)
    ap.add_argument("--test", type=int, default=10)
    ap.add_argument("--api", action="store_true",
                    help="through the public API: cgnn.GNN().predict_proba(a, b) with max_nb_points=None "
                         "(the scorer routes the long runs to the sample-sharded trainer)")
    ap.add_argument("--runs", type=int, default=1, help="--api: nb_runs (2 models each)")
    a = ap.parse_args()
    if a.api:
        return api(a)
    from cgnn_amd.engine.program import program_for_dag, program_for_pair
    from cgnn_amd.engine.sharded import SampleShardedTrainer, shard_range
    from cgnn_amd.parallel import dist as pdist
    from cgnn_amd.utils.graph import DirectedGraph
    from cgnn_amd.utils.philox import model_key
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        pdist.init_process_group("nccl")
    rank = pdist.rank()
    torch.cuda.set_device(pdist.local_rank())
    dev = torch.device("cuda", torch.cuda.current_device())
    rng = np.random.default_rng(0)
    x = rng.standard_normal((a.d, a.N)).astype(np.float32)
    x[1] += np.tanh(x[0])
    if a.d == 2:
        prog = program_for_pair(a.h)
    else:
        g = DirectedGraph()
        for k in range(a.d - 1):
            g.add("V%d" % k, "V%d" % (k + 1))
        prog = program_for_dag(g, a.h)
    r0, n = shard_range(a.N, rank, world)
    t0 = time.perf_counter()
    tr = SampleShardedTrainer([prog], [x[:, r0:r0 + n]], [model_key(0, "long")], a.h, dev, a.N)
    tr.train(2)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    t1 = time.perf_counter()
    tr.train(a.train)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    score = tr.evaluate(a.test)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    pairs = float(a.N) * 2 * a.N          # (row, column) pairs of the MMD per step
    if rank == 0:
        print(json.dumps({"bench": "cgnn_long_n", "N": a.N, "d": a.d, "h": a.h, "ranks": world,
                          "mmd_kernel": tr.kernel, "ms_per_train_step": round(1e3 * (t2 - t1) / a.train, 3),
                          "ms_per_eval_step": round(1e3 * (t3 - t2) / a.test, 3),
                          "mmd_pairs_per_s_train": round(pairs * a.train / (t2 - t1), 1),
                          "exp_evals_per_s_train": round(7 * pairs * a.train / (t2 - t1), 1),
                          "score": float(score[0]), "setup_s": round(setup, 2)}), flush=True)


def api(a):
    import cgnn
    from cgnn_amd.parallel import dist as pdist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        pdist.init_process_group("nccl")
    rng = np.random.default_rng(0)
    x = rng.standard_normal(a.N)
    y = np.tanh(x) + 0.3 * rng.standard_normal(a.N)
    kw = dict(nb_runs=a.runs, train_epochs=a.train, test_epochs=a.test, max_nb_points=None, h_layer_dim=a.h)
    cgnn.GNN().predict_proba(x[:4096], y[:4096], **dict(kw, train_epochs=2, test_epochs=1))   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = cgnn.GNN().predict_proba(x, y, **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if pdist.rank() == 0:
        steps = a.train + a.test
        print(json.dumps({"bench": "cgnn_long_n_api", "call": "cgnn.GNN().predict_proba", "N": a.N, "nb_runs": a.runs,
                          "models": 2 * a.runs, "train_epochs": a.train, "test_epochs": a.test, "ranks": world,
                          "seconds": round(dt, 3), "ms_per_step": round(1e3 * dt / steps, 3), "score": float(s),
                          "direction_correct": bool(s > 0)}), flush=True)


if __name__ == "__main__":
    main()
