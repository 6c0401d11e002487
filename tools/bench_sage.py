"""GraphSAGE mini-batch training throughput (GNN track, not in the reference).

    python tools/bench_sage.py --dataset ogbn-products --fanouts 15 10 --batch 1024 --epochs 2

Synthetic graph of the named dataset's shape; reports seeds/s and s/epoch
(sampling on a host thread overlapped with the GPU step) and the full-graph
validation accuracy."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="ogbn-products")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--fanouts", type=int, nargs="+", default=[15, 10])
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--max-batches", type=int, default=0, help="truncate the train split (quick runs)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic(a.dataset, seed=0, device="cuda:0", scale=a.scale)
    tr = SAGETrainer(g, hidden=a.hidden, fanouts=a.fanouts, batch_size=a.batch)
    if a.max_batches:
        tr.train_idx = tr.train_idx[:a.max_batches * a.batch]
    tr.train_epoch()                      # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.epochs):
        loss = tr.train_epoch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.epochs
    res = tr.evaluate()
    print(json.dumps({"bench": "sage_minibatch", "dataset": a.dataset, "n": g.n, "fanouts": a.fanouts,
                      "batch": a.batch, "seeds_per_epoch": int(len(tr.train_idx)), "s_per_epoch": dt,
                      "seeds_per_s": len(tr.train_idx) / dt, "train_loss": loss, **res}))


if __name__ == "__main__":
    main()
