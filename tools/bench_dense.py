"""Micro-benchmark of the fused dense GCN kernels (gnn_dense.hip) on the
ogbn-products shape: forward (AX W1 -> bias/ReLU/dropout -> W2, H1 not stored)
and the fused backward, at the given dropout rates.  One JSON line per kernel
and rate: time per launch and the MFMA rate of the products it performs.

    python tools/bench_dense.py [--rows 2449029] [--reps 20] [--p 0.5 0.0]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2449029)
    ap.add_argument("--F", type=int, default=100)
    ap.add_argument("--C", type=int, default=47)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--p", type=float, nargs="+", default=[0.5, 0.25, 0.1, 0.0])
    ap.add_argument("--aligned", action="store_true", help="row pitches of the headline: whole 128-B lines")
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    dev = torch.device("cuda", 0)
    n, F, C, HD = a.rows, a.F, a.C, a.hidden
    ldx, ldc = (F + 1 + 7) // 8 * 8, (C + 7) // 8 * 8
    if a.aligned:
        ldx, ldc = (F + 1 + 63) // 64 * 64, (C + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(0)
    AX = torch.randn(n, ldx, device=dev, generator=g).to(torch.bfloat16)
    dY2 = (torch.randn(n, ldc, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    W1 = torch.randn(F, HD, device=dev, generator=g) * 0.1
    b1 = torch.randn(HD, device=dev, generator=g) * 0.1
    W2 = torch.randn(HD, C, device=dev, generator=g) * 0.1
    dinv = torch.rand(n, device=dev, generator=g)
    Z2 = torch.empty(n, ldc, device=dev, dtype=torch.bfloat16)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    key = (12345, 678)
    fl_fwd = 2.0 * n * HD * (F + C)
    fl_bwd = 2.0 * n * HD * (2 * F + 2 * C)
    gpart = None
    for p in a.p:
        def fwd():
            ops.dense_fwd(AX, W1, b1, W2, dinv, None, Z2, F, p, key, 3)

        def bwd():
            nonlocal gpart
            _, _, _, gpart = ops.fused_bwd(AX, dY2, W1, b1, W2, n, F, p, key, 3, 0, gpart)
        for name, fn, fl in (("dense_fwd", fwd, fl_fwd), ("fused_bwd", bwd, fl_bwd)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ev0.record()
            for _ in range(a.reps):
                fn()
            ev1.record()
            torch.cuda.synchronize()
            ms = ev0.elapsed_time(ev1) / a.reps
            print(json.dumps({"kernel": name, "p": p, "rows": n, "ms": round(ms, 4),
                              "TFLOPs": round(fl / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
