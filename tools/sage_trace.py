"""Steady-state per-batch view of a GraphSAGE kernel trace (rocprofv3 --kernel-trace csv):
wall per batch, busy time per stream, the time both streams run kernels at once, and
the heaviest kernels; optionally the HIP API calls per batch (--api).

    python tools/sage_trace.py gpurun_out/r05_sage4/trace [--api]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith("sb_scanA")]
    per = 5                                       # scanA launches per batch (3 levels + 2 transposes)
    starts = first[::per]
    w0, w1 = starts[-190], starts[-10]
    nb = 180
    win = [r for r in rows if w0 <= int(r["Start_Timestamp"]) < w1]
    busy, names = collections.Counter(), collections.Counter()
    iv = collections.defaultdict(list)
    for r in win:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy[r["Stream_Id"]] += b - a
        names[(r["Stream_Id"], r["Kernel_Name"][:48])] += b - a
        iv[r["Stream_Id"]].append((a, b))

    def union(x):
        x = sorted(x)
        out = []
        for a, b in x:
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out

    u = {k: union(v) for k, v in iv.items()}
    tot = {k: sum(b - a for a, b in v) for k, v in u.items()}
    allu = union([tuple(x) for v in u.values() for x in v])
    any_busy = sum(b - a for a, b in allu)
    print("wall per batch us %.1f" % ((w1 - w0) / nb / 1e3))
    for k in sorted(tot):
        print("stream %s busy (union) per batch us %.1f  kernel-sum %.1f" % (k, tot[k] / nb / 1e3, busy[k] / nb / 1e3))
    print("any stream busy per batch us %.1f; both at once %.1f" % (any_busy / nb / 1e3,
                                                                     (sum(tot.values()) - any_busy) / nb / 1e3))
    for k, v in names.most_common(30):
        print("%7.1f %s" % (v / nb / 1e3, k))
    if "--api" in sys.argv:
        f = glob.glob(os.path.join(d, "*hip_api_trace.csv"))
        if f:
            api = [r for r in csv.DictReader(open(f[0])) if w0 <= int(r["Start_Timestamp"]) < w1]
            c = collections.Counter(r["Function"] for r in api)
            t = collections.Counter()
            for r in api:
                t[r["Function"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for k, v in c.most_common(20):
                print("%6.2f per batch %7.1f us/batch %s" % (v / nb, t[k] / nb / 1e3, k))


if __name__ == "__main__":
    main()
