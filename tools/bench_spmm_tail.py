"""How much of an SpMM launch is the tail of its longest rows?  On the headline graph
(ogbn-products shape, shuffled ids + the reorder pass) times the layer-1 aggregation
(F 100, 128-element pitch, L = 16) and the train-row layer-2 aggregation (F 47, 48-element
pitch, L = 8) over (a) the whole CSR, (b) the CSR with the rows longer than T emptied,
(c) those long rows only.  If (a) is well above (b) the launch waits for a few long rows
that one lane sub-group walks alone.

    python tools/bench_spmm_tail.py [--T 256] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _subset(rp, col, keep):
    """CSR with the rows where ``keep`` is False emptied (same row count)."""
    deg = (rp[1:] - rp[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(deg.numel(), device=rp.device), deg)
    sel = keep[rows]
    nd = torch.where(keep, deg, torch.zeros_like(deg))
    out = torch.zeros_like(rp, dtype=torch.int64)
    out[1:] = torch.cumsum(nd, 0)
    return out.to(torch.int32), col[sel].contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from cgnn_amd.gnn import ops
    from cgnn_amd.gnn.data import synthetic, reorder
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, id_order="shuffled")
    g, _ = reorder(g)
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
        return round(ev0.elapsed_time(ev1) / a.reps, 4)

    rp, col = g.rowptr, g.col
    deg = (rp[1:] - rp[:-1]).long()
    long_rows = deg > a.T
    X = torch.randn(g.n, 128, device=dev).to(torch.bfloat16)
    Y = torch.empty(g.n, 128, device=dev, dtype=torch.bfloat16)
    res = {"T": a.T, "n_long": int(long_rows.sum()), "max_deg": int(deg.max())}
    for name, (r, c) in (("l1_all", (rp, col)), ("l1_short", _subset(rp, col, ~long_rows)),
                         ("l1_long", _subset(rp, col, long_rows))):
        res[name + "_ms"] = timed(lambda: ops.spmm(r, c, X, 100, rscale=g.dinv, out=Y))
    # the train rows' layer-2 aggregation (compact CSR of the train rows, as gcn.py builds it)
    trows = torch.nonzero(g.mask == 1).flatten()
    lo, tdeg = rp[trows].long(), deg[trows]
    trp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
    trp[1:] = torch.cumsum(tdeg, 0)
    eid = torch.arange(int(trp[-1]), device=dev) + torch.repeat_interleave(lo - trp[:-1], tdeg)
    trp32, tcol = trp.to(torch.int32), col[eid].contiguous()
    tlong = tdeg > a.T // 2
    Z = torch.randn(g.n, 48, device=dev).to(torch.bfloat16)
    Z2 = torch.empty(trows.numel(), 48, device=dev, dtype=torch.float32)
    res["n_train_long"] = int(tlong.sum())
    for name, (r, c) in (("l2_all", (trp32, tcol)), ("l2_short", _subset(trp32, tcol, ~tlong)),
                         ("l2_long", _subset(trp32, tcol, tlong))):
        res[name + "_ms"] = timed(lambda: ops.spmm(r, c, Z, 47, out=Z2, out_dtype=torch.float32))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
