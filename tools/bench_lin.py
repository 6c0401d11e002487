"""Time the SAGE layer-0 dense kernels on their shapes: lin_fwd ([x[idx] | agg] @ W + b,
ReLU, dropout), lin_bwd_data and lin_bwd_weight, at several row counts, with and without
the gathered first operand and the dropout -- to see which part of a call is the work.

    python tools/bench_lin.py [--reps 20]
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
    ap.add_argument("--rows", type=int, nargs="+", default=[6000, 20000, 60000, 200000])
    ap.add_argument("--shape", choices=["sage", "arxiv"], default="sage",
                    help="arxiv: the 3-layer GCN's dense kernels at 169,343 rows (K 128 / 256 -> 256, 256 -> 40)")
    a = ap.parse_args()
    from cgnn_amd.gnn.linear import lin_bwd_data, lin_bwd_weight, lin_fwd
    dev = torch.device("cuda", 0)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(a.reps):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        return round(1000 * ev0.elapsed_time(ev1) / a.reps, 1)

    if a.shape == "arxiv":
        n, H, C = 169343, 256, 40
        x0 = torch.randn(n, 128, device=dev).to(torch.bfloat16)
        h = torch.randn(n, H, device=dev).to(torch.bfloat16)
        W0 = torch.randn(128, H, device=dev) / 11
        W1 = torch.randn(H, H, device=dev) / 16
        W2 = torch.randn(H, C, device=dev) / 16
        b = torch.randn(H, device=dev) / 10
        dinv = torch.rand(n, device=dev) + 0.5
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        y = torch.empty(n, H, device=dev, dtype=torch.bfloat16)
        lin_fwd(h, W1, b, relu=True, p=0.5, step=step, out=y)
        dY = torch.randn(n, H, device=dev).to(torch.bfloat16)
        dZ = torch.randn(n, C, device=dev).to(torch.bfloat16)
        dX = torch.empty(n, H, device=dev, dtype=torch.bfloat16)
        r = {"n": n}
        r["fwd_k128_us"] = timed(lambda: lin_fwd(x0, W0, b, relu=True, p=0.5, step=step, out=y))
        r["fwd_k256_us"] = timed(lambda: lin_fwd(h, W1, b, relu=True, p=0.5, step=step, out=y))
        r["fwd_k256_nodrop_us"] = timed(lambda: lin_fwd(h, W1, b, relu=True, out=dX))
        r["bwd_data_n256_us"] = timed(lambda: lin_bwd_data(dY, W1, H, Ym=y, mscale=2.0, rscale=dinv, out1=dX))
        r["bwd_data_n40_us"] = timed(lambda: lin_bwd_data(dZ, W2, H, rscale=dinv, out1=dX))
        print(json.dumps(r), flush=True)
        return
    F, N = 104, 256
    table = torch.randn(2449029, F, device=dev).to(torch.bfloat16)
    W = torch.randn(2 * F, N, device=dev) / 16
    b = torch.randn(N, device=dev) / 10
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    for n in a.rows:
        idx = torch.randint(0, table.shape[0], (n,), device=dev, dtype=torch.int32)
        xg = table[idx.long()].contiguous()
        agg = torch.randn(n, F, device=dev).to(torch.bfloat16)
        out = torch.empty(n, N, device=dev, dtype=torch.bfloat16)
        dY = torch.randn(n, N, device=dev).to(torch.bfloat16)
        r = {"n": n}
        r["fwd_gather_drop_us"] = timed(lambda: lin_fwd(table, W, b, x2=agg, K1=F, K2=F, relu=True, p=0.5, step=step,
                                                        idx1=idx, n=n, out=out))
        r["fwd_gather_us"] = timed(lambda: lin_fwd(table, W, b, x2=agg, K1=F, K2=F, relu=True, idx1=idx, n=n, out=out))
        r["fwd_plain_us"] = timed(lambda: lin_fwd(xg, W, b, x2=agg, K1=F, K2=F, relu=True, out=out))
        dhd = torch.empty(n, F, device=dev, dtype=torch.float32)
        dag = torch.empty(n, F, device=dev, dtype=torch.bfloat16)
        r["bwd_data_us"] = timed(lambda: lin_bwd_data(dY, W, F, F, Ym=out, mscale=2.0, out1=dhd, out2=dag))
        r["bwd_weight_gather_us"] = timed(lambda: lin_bwd_weight(table, dY, N, x2=agg, K1=F, K2=F, Ym=out, mscale=2.0,
                                                                 idx1=idx, n=n))
        r["bwd_weight_plain_us"] = timed(lambda: lin_bwd_weight(xg, dY, N, x2=agg, K1=F, K2=F, Ym=out, mscale=2.0))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
