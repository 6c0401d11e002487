"""GraphSAGE training-step time without the concurrent sampler (diagnostic only; not
the benchmark): products-sage3 as tools/bench_gnn_configs.py builds it, K batches
sampled once by the per-level DeviceSampler, then the fused training step replayed
over them on one stream.  Prints the level sizes and us per step; compare with the
pipelined epoch's us per batch to see what sampling beside the training costs.

    python tools/sage_train_only.py [--k 8] [--steps 192]
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
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--steps", type=int, default=192)
    a = ap.parse_args()
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn.sage import SAGETrainer
    from cgnn_amd.gnn.sampler import DeviceSampler
    dev = torch.device("cuda", 0)
    g, _ = reorder(synthetic("ogbn-products", seed=0, device=dev), seed=0)
    tr = SAGETrainer(g, hidden=256, layers=3, dropout=0.5, lr=0.003, fanouts=(15, 10, 5), batch_size=1024)
    t0 = time.perf_counter()
    tr.train_epoch()
    torch.cuda.synchronize()
    epoch_s = time.perf_counter() - t0
    nb = len(tr._batches())
    ds = DeviceSampler(g.rowptr, g.col, [15, 10, 5], 0)
    batches = tr._batches()[:a.k]
    cached = []
    for k, b in enumerate(batches):
        seeds = torch.as_tensor(b.astype(np.int32), device=dev)
        blocks, nodes_in = ds.sample(seeds, 7 + k)
        for blk in blocks:
            blk.transposed()
        labels = tr.y32[seeds.long()]
        cached.append((blocks, nodes_in.to(torch.int32), seeds, labels))
    sizes = [[(blk.n_dst, blk.n_src, int(blk.col.numel())) for blk in c[0]] for c in cached[:2]]
    for c in cached:
        tr._step(c[0], c[1], c[2], c[3])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.steps):
        c = cached[s % len(cached)]
        tr._step(c[0], c[1], c[2], c[3])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"train_only_us_per_step": round(1e6 * dt, 1),
                      "pipelined_epoch_us_per_batch": round(1e6 * epoch_s / nb, 1), "batches_per_epoch": nb,
                      "blocks_input_first_(n_dst,n_src,nnz)": sizes}))


if __name__ == "__main__":
    main()
