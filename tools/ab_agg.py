"""A/B timing of the headline GCN's layer-1 forward on the ogbn-products shape (synthetic,
reorder pass, the training CSR of the train-neighbour rows): the layer-1 ``spmm`` and
``dense_fwd`` as two kernels against the fused ``agg_fwd`` (HIP events, median of
``--iters``).  Run once per build (``CGNN_HIP_LIB=<variant .so>`` from
tools/build_variant.sh).  Development tool; the shipped numbers come from bench.py."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cgnn_amd.gnn import ops  # noqa: E402
from cgnn_amd.gnn.data import synthetic  # noqa: E402
from cgnn_amd.gnn.gcn import GCNTrainer  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1), round(ts[0], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--only-agg", action="store_true")
    ap.add_argument("--only-spmm", action="store_true")
    ap.add_argument("--only-ell", action="store_true", help="the backward's train-column aggregation (spmm_ell)")
    a = ap.parse_args()
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=a.scale)
    tr = GCNTrainer(g, hidden=256, rank=0, world=1, reorder=True, fuse_agg=True)
    del g
    rp, col = tr._l1
    n, F = tr.nloc, tr.F
    key, step = tr.key, tr.step_t
    res = {"lib": os.environ.get("CGNN_HIP_LIB", "default"), "n": n, "nnz_l1": int(col.numel())}

    def spmm():
        ops.spmm(rp, col, tr.Xs, F, rscale=tr.dinv, out=tr.AX, unit_col=F)

    def dense():
        ops.dense_fwd(tr.AX, tr.W1, tr.b1, tr.W2, tr.dinv, None, tr.Z2loc[:n], F, 0.5, key, step, 0, kimg=tr._kimg)

    def agg():
        ops.agg_fwd(rp, col, tr.Xs, tr.AX, tr.W1, tr.b1, tr.W2, tr.dinv, tr.Z2loc, F, 0.5, key, step, 0,
                    kimg=tr._kimg, queue=tr._agg_queue)

    def ell():
        ops.spmm_ell(tr._ell_T, tr.col_T, tr.Gc, tr.C, rscale=tr.dinv, out=tr.dY2)

    todo = (("agg", agg),) if a.only_agg else (("spmm", spmm),) if a.only_spmm else (("ell", ell),) if a.only_ell \
        else (("spmm", spmm), ("dense", dense), ("agg", agg))
    for name, fn in todo:
        res[name + "_us"], res[name + "_min_us"] = timed(fn, a.iters)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
