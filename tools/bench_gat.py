"""Full-graph GAT training throughput (GNN track, not in the reference).

    python tools/bench_gat.py --dataset ogbn-products --heads 4 --head-dim 32 --steps 5

Synthetic graph of the dataset's shape; reports ms per epoch (forward + backward +
Adam over the whole graph) and accuracies."""
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
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--head-dim", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--unfused", action="store_true", help="autograd model + hipBLASLt projections (A/B)")
    ap.add_argument("--reorder", choices=["lp-cm", "none"], default="lp-cm",
                    help="framework locality pass at setup (the synthetic ids are shuffled)")
    a = ap.parse_args()
    import torch
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import GATTrainer
    g = synthetic(a.dataset, seed=0, device="cuda:0", scale=a.scale)
    t0 = time.perf_counter()
    tr = GATTrainer(g, heads=a.heads, head_dim=a.head_dim, fused=False if a.unfused else None,
                    reorder=a.reorder != "none")
    setup = time.perf_counter() - t0
    for _ in range(a.warmup):
        tr.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = tr.train_step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    res = tr.evaluate()
    print(json.dumps({"bench": "gat_fullgraph", "dataset": a.dataset, "n": g.n, "nnz": g.nnz,
                      "heads": a.heads, "head_dim": a.head_dim, "ms_per_epoch": 1e3 * dt,
                      "epochs_per_s": 1.0 / dt, "train_loss": float(loss), "fused": tr.fused is not None,
                      "reordered": a.reorder != "none", "trainer_setup_s": round(setup, 2),
                      **res}))


if __name__ == "__main__":
    main()
