"""Layer-1 SpMM cost against the gathered row's width and pitch, on the headline graph
(ogbn-products shape, shuffled ids + the reorder pass, as bench.py builds it).  Each
variant gathers F bf16 columns from rows of pitch ``ld``: does the time follow the
64-B sectors a gather touches (F 100 touches four of a 256-B row, F 96 three), the
128-B lines, or the row count?

    python tools/bench_spmm_width.py [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="100:128,96:96")
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    from cgnn_amd.gnn.data import synthetic, reorder
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, id_order="shuffled")
    g, _ = reorder(g)
    n, nnz = g.n, g.nnz
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for v in a.variants.split(","):
        F, ld = (int(t) for t in v.split(":"))
        X = torch.randn(n, ld, device=dev).to(torch.bfloat16)
        Y = torch.empty(n, max(ld, 8), device=dev, dtype=torch.bfloat16)

        def run():
            ops.spmm(g.rowptr, g.col, X, F, rscale=g.dinv, out=Y)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.reps):
            run()
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / a.reps
        print(json.dumps({"F": F, "ld": ld, "ms": round(ms, 4), "nnz": nnz,
                          "x_MB": round(n * ld * 2 / 1e6, 1)}), flush=True)
        del X, Y
    # the split table (ops.SplitRows) of the 100 features against the 256-B rows
    X = torch.randn(n, 128, device=dev).to(torch.bfloat16)
    S = ops.SplitRows(X, 100)
    Y0 = torch.empty(n, 104, device=dev, dtype=torch.bfloat16)
    Y1 = torch.empty_like(Y0)
    for name, tab, Y in (("dense128", X, Y0), ("split96+8", S, Y1), ("dense128", X, Y0), ("split96+8", S, Y1)):
        def run():
            ops.spmm(g.rowptr, g.col, tab, 100, rscale=g.dinv, out=Y, unit_col=100)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.reps):
            run()
        ev1.record()
        torch.cuda.synchronize()
        print(json.dumps({"table": name, "F": 100, "ms": round(ev0.elapsed_time(ev1) / a.reps, 4)}), flush=True)
    print(json.dumps({"split_bitwise_equal": bool(torch.equal(Y0.view(torch.int16), Y1.view(torch.int16)))}))


if __name__ == "__main__":
    main()
