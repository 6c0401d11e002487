"""Where a GraphSAGE mini-batch epoch's wall time goes on the host (products-sage3 shape,
pipelined sampler): the time the Python thread spends waiting for each batch's sampling
(``resolve``), enqueuing the training step (``_step``), and the epoch's wall time.  If
enqueue time ~ wall time the loop is launch-bound; if the resolve wait dominates, the
side-stream sampler is the critical path.

    python tools/sage_host.py [--scale 1.0] [--epochs 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args()
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn import sage as sage_mod
    from cgnn_amd.gnn.sampler import SampledBatch
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, scale=a.scale)
    g, _ = reorder(g)
    tr = sage_mod.SAGETrainer(g, hidden=256, layers=3, dropout=0.5, lr=0.003, fanouts=(15, 10, 5),
                              batch_size=1024, seed=0)
    acc = {"resolve": 0.0, "step": 0.0, "n": 0}
    orig_resolve, orig_step = SampledBatch.resolve, tr._step

    def resolve(self):
        t = time.perf_counter()
        r = orig_resolve(self)
        acc["resolve"] += time.perf_counter() - t
        return r

    def step(*args, **kw):
        t = time.perf_counter()
        r = orig_step(*args, **kw)
        acc["step"] += time.perf_counter() - t
        acc["n"] += 1
        return r

    SampledBatch.resolve = resolve
    tr._step = step
    tr.train_epoch()                       # warm-up
    torch.cuda.synchronize()
    for e in range(a.epochs):
        acc.update(resolve=0.0, step=0.0, n=0)
        t0 = time.perf_counter()
        tr.train_epoch()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(json.dumps({"epoch": e, "wall_ms": round(wall * 1e3, 2), "batches": acc["n"],
                          "resolve_wait_ms": round(acc["resolve"] * 1e3, 2),
                          "step_enqueue_ms": round(acc["step"] * 1e3, 2),
                          "per_batch_us": {"wall": round(wall * 1e6 / max(acc["n"], 1), 1),
                                           "resolve": round(acc["resolve"] * 1e6 / max(acc["n"], 1), 1),
                                           "enqueue": round(acc["step"] * 1e6 / max(acc["n"], 1), 1)}}),
              flush=True)


if __name__ == "__main__":
    main()
