"""Summarise rocprofv3 CSV output (``--output-format csv``) per kernel.

    python tools/pmc_summary.py --trace gpurun_out/prof/trace --pmc gpurun_out/prof/pmc_a \
        gpurun_out/prof/pmc_b [--top 12] [--match spmm]

* ``--trace``: a ``--kernel-trace`` run -> calls and total / mean time per kernel;
* ``--pmc``:   one or more ``--pmc`` runs (one counter set each) -> per-kernel sums.

Derived columns (when the counters are present):
  L2 hit        TCC_HIT / (TCC_HIT + TCC_MISS)
  fetch MB      FETCH_SIZE (KB) x 1024 per dispatch; on gfx950 FETCH_SIZE counts a
                wide coalesced stream at half its bytes (MI355X_MICROARCH.md, HBM),
                so ``x2`` is the upper bound of the true memory-side read traffic
  TB/s          fetch bytes / mean kernel time, both the raw and the x2 figure
  VALU, WAIT    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, SQ_WAIT_ANY / SQ_WAVE_CYCLES
Counters are summed over all dispatches of a kernel name and divided by the
dispatch count.  Prints a markdown table.
"""
import argparse
import collections
import csv
import glob
import os


def _rows(path, suffix):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*" + suffix), recursive=True)
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def trace_times(path):
    t = collections.defaultdict(list)
    for r in _rows(path, "kernel_trace.csv"):
        t[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return t


def counters(paths):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in _rows(p, "counter_collection.csv"):
            k = r["Kernel_Name"]
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add((p, r.get("Dispatch_Id") or r.get("Correlation_Id")))
    out = {}
    for k, cs in sums.items():
        out[k] = {c: v / max(len(disp[(k, c)]), 1) for c, v in cs.items()}
    return out


def short(name, n=70):
    name = name.replace("void ", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    times = trace_times(a.trace) if a.trace else {}
    pmc = counters(a.pmc)
    names = list(times) or list(pmc)
    tot = sum(sum(v) for v in times.values()) or 1
    names.sort(key=lambda k: -sum(times.get(k, [0])))
    names = [k for k in names if a.match in k][:a.top]
    print("| kernel | calls | mean us | % time | L2 hit | fetch MB | TB/s (raw / x2) | VALU | WAIT |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in names:
        ts = times.get(k, [])
        mean_us = sum(ts) / len(ts) / 1e3 if ts else float("nan")
        c = pmc.get(k, {})
        hit = c.get("TCC_HIT_sum", c.get("TCC_HIT"))
        miss = c.get("TCC_MISS_sum", c.get("TCC_MISS"))
        l2 = "%.3f" % (hit / (hit + miss)) if hit is not None and miss is not None and hit + miss > 0 else "-"
        fetch = c.get("FETCH_SIZE")
        fmb = "%.1f" % (fetch * 1024 / 1e6) if fetch is not None else "-"
        bw = ("%.2f / %.2f" % (fetch * 1024 / (mean_us * 1e-6) / 1e12, 2 * fetch * 1024 / (mean_us * 1e-6) / 1e12)
              if fetch is not None and ts else "-")
        wc = c.get("SQ_WAVE_CYCLES")
        valu = "%.2f" % (c["SQ_ACTIVE_INST_VALU"] / wc) if wc and "SQ_ACTIVE_INST_VALU" in c else "-"
        wait = "%.2f" % (c["SQ_WAIT_ANY"] / wc) if wc and "SQ_WAIT_ANY" in c else "-"
        print("| %s | %d | %.1f | %.1f | %s | %s | %s | %s | %s |" % (
            short(k), len(ts), mean_us, 100 * sum(ts) / tot, l2, fmb, bw, valu, wait))


if __name__ == "__main__":
    main()
