"""A/B of the two Fourier-feature MMD forms (rff_kernels.hip): the register / MFMA form
compiled per padded width D (up to 256) against the wide form (theta scratch image, any
D), on the CGNN shapes (F = 7 x 100 features, N = 500 samples), train mode (loss
partials + gradient).  HIP events, median of 20 launches.

    python tools/ab_rff.py [--R 32 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, nargs="+", default=[32, 256])
    ap.add_argument("--N", type=int, default=500)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    from cgnn_amd import native
    hip = native.hip()
    st = torch.cuda.current_stream().cuda_stream
    k, N = a.k, a.N
    F = 7 * k
    for R in a.R:
        for D in (24, 64, 128, 160, 192, 224, 256):
            xhat = torch.randn(R, D, N, device="cuda") * 0.5
            data = torch.randn(R, D, N, device="cuda") * 0.5
            keys = torch.randint(0, 2**31 - 1, (R, 2), dtype=torch.int32, device="cuda")
            step = torch.zeros(2, dtype=torch.int32, device="cuda")
            W = torch.zeros(R, F, D + 1, device="cuda")
            hip.rff_freqs(W.data_ptr(), keys.data_ptr(), step.data_ptr(), 0, k, D, 7, D, R, st)
            scratch = torch.zeros(hip.rff_wide_scratch_floats(N, F, R), device="cuda")
            diff = torch.zeros(R, F, device="cuda")
            lp = torch.zeros(R, (F + 255) // 256, device="cuda")
            gp = torch.zeros(1, R, D, N, device="cuda")
            res = {"R": R, "D": D, "N": N, "F": F}
            for name, wide in (("narrow_us", 0), ("wide_us", 1)):
                res[name] = round(timed(lambda: hip.rff_fwd_bwd(
                    0, xhat.data_ptr(), data.data_ptr(), W.data_ptr(), diff.data_ptr(), lp.data_ptr(), gp.data_ptr(),
                    N, D, F, R, k, (2.0 / k) ** 0.5, st, scratch=scratch.data_ptr(), force_wide=wide)), 1)
            print(json.dumps(res), flush=True)
            del xhat, data, W, scratch, gp
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
