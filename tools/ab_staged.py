"""A/B of the level-scheduled generator kernels (cgnn_staged.hip) on one d-variable
batch: waves per block x sample-state placement, forward and backward timed alone.

    python tools/ab_staged.py --d 200 --edges 400 --R 256 --n 500 --h 20
Prints one JSON line per (kernel, W, placement): median / min microseconds."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--edges", type=int, default=400)
    ap.add_argument("--R", type=int, default=256)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--h", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="kernel:W:placement, e.g. bwd:4:2 (profiling runs)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from bench_cgnn_batch import random_dag_program
    from cgnn_amd import native
    from cgnn_amd.engine.batch import DeviceTrainer
    from cgnn_amd.utils.philox import model_key
    hip = native.hip()
    prog = random_dag_program(a.d, a.edges, a.h, 0, 0)
    data = np.random.default_rng(1).normal(size=(a.d, a.n)).astype(np.float32)
    tr = DeviceTrainer([prog] * a.R, [data] * a.R, [model_key(0, r) for r in range(a.R)], a.h, "cuda:0",
                       graph_chunk=0, generator="staged")
    tr.run(3, 1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    R, N, D, d, H, P = a.R, a.n, tr.D, a.d, a.h, tr.P
    T = hip.staged_tiles(N)
    gradp = (torch.randn(1, R, D, N, device="cuda") * 1e-3).contiguous()
    gp = torch.zeros(R, T, P, device="cuda")
    dxs = torch.zeros(R, d, N, device="cuda")
    xh = torch.zeros_like(tr.xhat)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return ts[len(ts) // 2], ts[0]

    print(json.dumps({"max_in": int(tr.max_in), "plan_W": tr.stage_w,
                      "plan": list(hip.staged_plan(d, H, int(tr.max_in), tr.stage_w, tr.prog_stride + tr.sched_stride))}))
    only = a.only.split(":") if a.only else None
    for W in (1, 2, 4, 8):
        if only and int(only[1]) != W:
            continue
        for force in (0, 1):
            if only and (only[0] != "fwd" or int(only[2]) != force):
                continue
            try:
                med, mn = timeit(lambda: hip.gen_fwd_staged(
                    tr.prog.data_ptr(), tr.prog_stride, tr.sched.data_ptr(), tr.sched_stride, tr.params.data_ptr(),
                    P, tr.data.data_ptr(), xh.data_ptr(), tr.noise.data_ptr(), tr.NS, tr.xnorm.data_ptr(), N, D, d,
                    H, int(tr.max_in), R, W, st, force=force))
                print(json.dumps({"kernel": "fwd", "W": W, "xg": force, "med_us": round(med, 1), "min_us": round(mn, 1)}))
            except RuntimeError as e:
                print(json.dumps({"kernel": "fwd", "W": W, "xg": force, "skip": str(e)[:60]}))
        for force in (0, 1, 2):
            if only and (only[0] != "bwd" or int(only[2]) != force):
                continue
            try:
                med, mn = timeit(lambda: hip.gen_bwd_staged(
                    tr.prog.data_ptr(), tr.prog_stride, tr.sched.data_ptr(), tr.sched_stride, tr.params.data_ptr(),
                    P, tr.xhat.data_ptr(), tr.noise.data_ptr(), tr.NS, gradp.data_ptr(), 1, R, N, D, d, H,
                    int(tr.max_in), W, gp.data_ptr(), dxs.data_ptr(), st, force=force))
                print(json.dumps({"kernel": "bwd", "W": W, "place": force, "med_us": round(med, 1), "min_us": round(mn, 1)}))
            except RuntimeError as e:
                print(json.dumps({"kernel": "bwd", "W": W, "place": force, "skip": str(e)[:60]}))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
