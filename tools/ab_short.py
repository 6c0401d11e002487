"""A/B of the GraphSAGE backward's transposed aggregation (products-sage3 shapes): the
one-row-per-sub-group spmm_kernel against spmm_short_kernel (4 rows per sub-group), on
the transposed blocks the pipelined sampler builds for a real batch.  HIP events,
median of 20 launches per form.

    python tools/ab_short.py [--scale 1.0]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=20):
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
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn.sampler import PipelinedSampler
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, scale=a.scale)
    g, _ = reorder(g)
    ps = PipelinedSampler(g.rowptr, g.col, [15, 10, 5], 1024, seed=0)
    rng = np.random.default_rng(0)
    seeds = torch.as_tensor(rng.choice(g.n, 1024, replace=False).astype(np.int32), device=dev)
    blocks, _ = ps.enqueue(seeds, 1).resolve()
    torch.cuda.synchronize()
    for k in (2, 1):                       # the backward's transposed aggregations
        blk = blocks[k]
        rp_t, col_t = blk.transposed()
        nd, ns = blk.n_dst, blk.n_src
        dagg = torch.randn(nd, 256, device=dev).to(torch.bfloat16)
        dhd = torch.randn(nd, 256, device=dev)
        out = torch.empty(ns, 256, dtype=torch.bfloat16, device=dev)
        res = {"block": k, "n_src": ns, "n_dst": nd, "nnz": int(col_t.numel())}
        deg = (rp_t[1:] - rp_t[:-1]).cpu().numpy()
        res["deg_max"] = int(deg.max())
        res["deg_p"] = {q: float(np.percentile(deg, q)) for q in (50, 90, 99, 99.9)}
        res["rows_ge_32"] = int((deg >= 32).sum())
        res["nnz_in_rows_ge_32"] = int(deg[deg >= 32].sum())
        outs = {}
        for name, sr in (("row", False), ("short", True)):
            f = lambda: ops.spmm(rp_t, col_t, dagg, 256, cscale=blk.inv_deg, init=dhd, init_rows=nd, out=out,
                                 short_rows=sr)
            f()
            torch.cuda.synchronize()
            res[name + "_us"] = round(timed(f), 1)
            outs[name] = out.clone()
        res["bitwise_equal"] = bool(torch.equal(outs["row"], outs["short"]))
        # which epilogue / gather option costs what
        for cs in (False, True):
            for ini in (False, True):
                for name, sr in (("row", False), ("short", True)):
                    f = lambda: ops.spmm(rp_t, col_t, dagg, 256, cscale=blk.inv_deg if cs else None,
                                         init=dhd if ini else None, init_rows=nd if ini else None, out=out,
                                         short_rows=sr)
                    res["%s_cs%d_init%d_us" % (name, cs, ini)] = round(timed(f), 1)
        # calibration: the same output written by a fill, and read + written by a copy
        res["fill_us"] = round(timed(lambda: out.fill_(1.0)), 1)
        src = out.clone()
        res["copy_us"] = round(timed(lambda: out.copy_(src)), 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
