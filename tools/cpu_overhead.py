"""Host-side cost of one GCN training epoch: wall time of train_step() calls when the
GPU is kept busy (enqueue-bound check for small per-rank epochs at 8 GPUs), measured
on the headline shape scaled to one rank's share (``--scale 1/8``) and full size."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=a.scale)
    tr = GCNTrainer(g, hidden=256, reorder=True)
    for _ in range(5):
        tr.train_step()
    torch.cuda.synchronize()
    # host cost per step: enqueue K steps back to back with the GPU idle at the start,
    # the queue deep enough that the host never waits
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(json.dumps({"scale": a.scale, "nodes": g.n, "host_ms_per_step": 1e3 * t_enq / a.steps,
                      "gpu_ms_per_step": 1e3 * t_all / a.steps}))


if __name__ == "__main__":
    main()
