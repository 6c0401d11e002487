"""A/B of the headline's layer-1 aggregation AX = D^-1/2 (A+I) Xs on the ogbn-products
shape (shuffled ids + the framework's reorder pass, as bench.py): one launch over the
whole 256-B rows (16 lanes per row) vs column slabs (``ops.spmm(slab=...)``: one launch
per 64-column slab, 8 lanes per row, each gathering one 128-B line per edge).  Checks
that every form gives the same bits, prints one JSON line per form (interleaved rounds).

    python tools/ab_spmm_slab.py [--scale 1.0] [--reps 20] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--slabs", default="0,64,32")
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    from cgnn_amd.gnn.data import synthetic, reorder
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, scale=a.scale)
    g, _ = reorder(g)
    n, F, ld = g.n, 100, 128
    X = torch.zeros(n, ld, device=dev, dtype=torch.bfloat16)
    X[:, :F] = torch.randn(n, F, device=dev).to(torch.bfloat16)
    slabs = [int(s) for s in a.slabs.split(",")]
    outs = {s: torch.empty(n, ld, device=dev, dtype=torch.bfloat16) for s in slabs}
    for s in slabs:
        ops.spmm(g.rowptr, g.col, X, F, rscale=g.dinv, out=outs[s], unit_col=F, slab=s)
    torch.cuda.synchronize()
    for s in slabs[1:]:
        assert torch.equal(outs[s], outs[slabs[0]]), "slab %d differs" % s
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {s: [] for s in slabs}
    for _ in range(a.rounds):
        for s in slabs:
            for _ in range(2):
                ops.spmm(g.rowptr, g.col, X, F, rscale=g.dinv, out=outs[s], unit_col=F, slab=s)
            torch.cuda.synchronize()
            ev0.record()
            for _ in range(a.reps):
                ops.spmm(g.rowptr, g.col, X, F, rscale=g.dinv, out=outs[s], unit_col=F, slab=s)
            ev1.record()
            torch.cuda.synchronize()
            res[s].append(ev0.elapsed_time(ev1) / a.reps)
    for s in slabs:
        print(json.dumps({"slab": s, "ms": [round(v, 4) for v in res[s]], "min_ms": round(min(res[s]), 4),
                          "nnz": g.nnz, "bitwise_equal": True}), flush=True)


if __name__ == "__main__":
    main()
