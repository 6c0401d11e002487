"""SpMM micro-benchmark on the ogbn-products shape (the three sparse passes of
the headline GCN epoch): gathered-row widths 100 (layer-1 features) and 47
(layer-2 logits / their gradient), bf16, with the row pitch either packed to
8 elements or padded to whole 128-B lines.  Prints one JSON line per variant:
time per launch and the effective gather rate nnz * row_bytes / t.

    python tools/bench_spmm.py [--scale 1.0] [--reps 20]
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
    ap.add_argument("--dataset", default="ogbn-products")
    ap.add_argument("--homophily", type=float, default=0.8)
    ap.add_argument("--id-order", default="banded", choices=["banded", "shuffled"])
    ap.add_argument("--reorder", action="store_true", help="framework locality pass first")
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    from cgnn_amd.gnn.data import synthetic, reorder
    dev = torch.device("cuda", 0)
    g = synthetic(a.dataset, seed=0, device=dev, scale=a.scale, homophily=a.homophily, id_order=a.id_order)
    if a.reorder:
        g, _ = reorder(g)
    n, nnz = g.n, g.nnz
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for F, ld in ((100, 104), (100, 128), (47, 48), (47, 64)):
        X = torch.randn(n, ld, device=dev).to(torch.bfloat16)
        Y = torch.empty(n, ld, device=dev, dtype=torch.bfloat16)

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
        row_b = F * 2
        print(json.dumps({"F": F, "ld": ld, "ms": round(ms, 4), "nnz": nnz,
                          "gather_TBps": round(nnz * row_b / ms / 1e9, 3),
                          "line_TBps": round(nnz * ld * 2 / ms / 1e9, 3),
                          "x_MB": round(n * ld * 2 / 1e6, 1)}), flush=True)
        del X, Y
    # the fused layer-2 aggregate + cross-entropy (train mode, compact gradient)
    C, ld = 47, 48
    Z = (torch.randn(n, ld, device=dev) * 0.1).to(torch.bfloat16)
    bias = torch.zeros(C, device=dev)
    train = g.mask == 1
    gslot = torch.where(train, torch.cumsum(train.int(), 0) - 1, torch.full_like(g.y, -1)).to(torch.int32)
    G = torch.empty(int(train.sum()), ld, device=dev, dtype=torch.bfloat16)
    for mode in (0, 1):
        def run_ce():
            ops.spmm_ce(g.rowptr, g.col, Z, C, g.dinv, bias, g.y, g.mask, 1e-6, mode=mode,
                        G=G if mode == 0 else None, gslot=gslot if mode == 0 else None)
        for _ in range(3):
            run_ce()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.reps):
            run_ce()
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / a.reps
        print(json.dumps({"kernel": "spmm_ce", "mode": mode, "C": C, "ld": ld, "ms": round(ms, 4),
                          "gather_TBps": round(nnz * C * 2 / ms / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
