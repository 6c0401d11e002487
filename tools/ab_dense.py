"""A/B timing of the headline GCN's fused dense kernels on the ogbn-products shape
(2,449,029 rows, 100 features + ones column, hidden 256, 47 classes, p = 1/2), random
operands, no graph: only ``gcn_dense_fwd`` and ``gcn_fused_bwd`` are timed (HIP events,
median of ``--iters``).  Run once per build (``CGNN_HIP_LIB=<variant .so>, built by tools/build_variant.sh``) and compare
the JSON lines.  Development tool; the shipped numbers come from bench.py."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cgnn_amd import native  # noqa: E402
from cgnn_amd.gnn import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2449029)
    ap.add_argument("--ldx", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, F, HD, C, ldc = a.n, 100, 256, 47, 48
    g = torch.Generator(device=dev).manual_seed(0)
    AX = torch.zeros(n, a.ldx, dtype=torch.bfloat16, device=dev)
    AX[:, :F] = (torch.randn(n, F, device=dev, generator=g) * 0.3).to(torch.bfloat16)
    AX[:, F] = 1
    dY2 = torch.zeros(n, ldc, dtype=torch.bfloat16, device=dev)
    dY2[:, :C] = (torch.randn(n, C, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    W1 = torch.randn(F, HD, device=dev, generator=g) * 0.1
    b1 = torch.randn(HD, device=dev, generator=g) * 0.01
    W2 = torch.randn(HD, C, device=dev, generator=g) * 0.1
    dinv = torch.rand(n, device=dev, generator=g) + 0.5
    Z2 = torch.zeros(n, ldc, dtype=torch.bfloat16, device=dev)
    kimg = ops.keep_image(n, HD, dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    hip = native.hip()
    nb, width = hip.gnn_fused_bwd_blocks(n), hip.gnn_fused_bwd_width(F + 1)
    gpart = torch.empty(nb, HD, width, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def fwd():
        ops.dense_fwd(AX, W1, b1, W2, dinv, None, Z2, F, a.p, (1, 2), step, 0, kimg=kimg)

    def bwd():
        rc = hip.gnn_fused_bwd(AX.data_ptr(), dY2.data_ptr(), W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                               kimg.data_ptr(), gpart.data_ptr(), n, F, a.ldx, HD, C, ldc, a.p, st)
        assert rc == 0, rc

    res = {"lib": os.environ.get("CGNN_HIP_LIB", "default")}
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        res[name + "_us"] = round(ts[len(ts) // 2], 1)
        res[name + "_min_us"] = round(ts[0], 1)
    res["gpart_checksum"] = float(gpart.double().sum().item())
    res["z2_checksum"] = float(Z2.double().sum().item())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
