"""Fractions of the other ranks' rows a rank receives per training epoch: the full
layer-2 halo (every row's sources) vs the training halo (the train rows' sources), on
the reordered ogbn-products shape, for 2 / 4 / 8 ranks (CPU only; ranks 0 and world/2
averaged).  Output: profiles/r02_l2rows/halo_fractions_cpu.log.

    python tools/halo_fractions.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cgnn_amd.gnn.data import partition_rows, reorder, synthetic  # noqa: E402


def main():
    t = time.time()
    g = synthetic("ogbn-products", seed=0)
    g, _ = reorder(g, seed=0)
    print("gen+reorder", time.time() - t, flush=True)
    for world in (2, 4, 8):
        fr_full, fr_tr = [], []
        for r in (0, world // 2):
            r0, r1, per, rp, col = partition_rows(g, r, world)
            col = col.long()
            rows = torch.repeat_interleave(torch.arange(r1 - r0), (rp[1:] - rp[:-1]).long())
            rem = (col < r0) | (col >= r1)
            tr = (g.mask[r0:r1] == 1)[rows]
            nrem = g.n - (r1 - r0)
            fr_full.append(torch.unique(col[rem]).numel() / nrem)
            fr_tr.append(torch.unique(col[rem & tr]).numel() / nrem)
        print(world, "full halo %.3f" % (sum(fr_full) / 2), "train halo %.3f" % (sum(fr_tr) / 2), flush=True)


if __name__ == "__main__":
    main()
