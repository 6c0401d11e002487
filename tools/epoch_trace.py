"""One steady-state training epoch out of a rocprofv3 kernel trace of bench.py: the
dispatches from the k-th training forward (the layer-1 ``spmm_kernel`` before a
``gcn_dense_fwd``) up to the next one, with durations and the gaps between them.

    python tools/epoch_trace.py <run_kernel_trace.csv> [k]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fw = [i for i, r in enumerate(rows) if "gcn_dense_fwd" in r["Kernel_Name"]]
    if len(fw) <= k + 1:
        sys.exit("only %d dense forwards in the trace" % len(fw))
    # the epoch starts with its layer-1 SpMM: back up from the forward to the previous spmm
    def start(i):
        while i > 0 and "spmm_kernel" not in rows[i]["Kernel_Name"]:
            i -= 1
        return i
    a, b = start(fw[k]), start(fw[k + 1])
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print("%9.1f us  +%6.1f  %8.1f us  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3, (e - s) / 1e3,
                                                r["Kernel_Name"][:90]))
        prev_end = e
    span = int(rows[b]["Start_Timestamp"]) - t0
    print("epoch span %.1f us, kernel busy %.1f us, %d dispatches" % (span / 1e3, busy / 1e3, b - a))


if __name__ == "__main__":
    main()
