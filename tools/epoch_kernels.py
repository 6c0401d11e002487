"""Ordered dispatch list of one steady-state epoch from a rocprofv3 kernel trace: the
dispatches from the k-th ``gcn_dense_fwd`` launch up to the next one (any form of the
GCN epoch, one-GPU or multi-rank), with durations, the gaps between them and a count
per kernel name (fills / copies included).

    python tools/epoch_kernels.py <run_kernel_trace.csv> [k]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fw = [i for i, r in enumerate(rows) if "gcn_dense_fwd" in r["Kernel_Name"]]
    if len(fw) <= k + 1:
        sys.exit("only %d dense forwards in the trace" % len(fw))
    a, b = fw[k], fw[k + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    count = collections.Counter()
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        count[name[:60]] += 1
        print("%9.1f us  +%6.1f  %8.1f us  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3, (e - s) / 1e3, name[:100]))
        prev_end = e
    span = int(rows[b]["Start_Timestamp"]) - t0
    print("epoch span %.1f us, %d dispatches" % (span / 1e3, b - a))
    for name, c in count.most_common():
        print("%4d  %s" % (c, name))


if __name__ == "__main__":
    main()
