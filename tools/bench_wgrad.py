"""Time the split-K weight gradient (lin_bwd_weight: dW = [X1 | X2]^T (dY * m), db) on the
shapes the GNN models hand it.

    python tools/bench_wgrad.py [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [  # name, n, K1, K2, N, masked
    ("sage_l1", 200000, 104, 104, 256, True),
    ("sage_hidden", 100000, 256, 256, 256, True),
    ("gat_products", 2449029, 104, 0, 256, False),
    ("arxiv_hidden", 169343, 256, 0, 256, True),
    ("gcn_deep_out", 169343, 256, 0, 40, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from cgnn_amd.gnn.linear import lin_bwd_weight
    dev = torch.device("cuda", 0)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for name, n, K1, K2, N, masked in SHAPES:
        x1 = torch.randn(n, K1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(n, K2, device=dev).to(torch.bfloat16) if K2 else None
        ldd = (N + 7) // 8 * 8
        dY = torch.randn(n, ldd, device=dev).to(torch.bfloat16)
        Ym = torch.relu(torch.randn(n, ldd, device=dev)).to(torch.bfloat16) if masked else None
        fn = lambda: lin_bwd_weight(x1, dY, N, x2=x2, K1=K1, Ym=Ym, mscale=2.0 if masked else 1.0)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.reps):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(1000 * ev0.elapsed_time(ev1) / a.reps, 1)
        del x1, x2, dY, Ym
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
