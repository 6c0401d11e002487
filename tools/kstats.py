"""Top kernels of a rocprofv3 ``--stats --output-format csv`` run (``*_kernel_stats.csv``):
calls, average and share, names shortened to the template.

    python tools/kstats.py gpurun_out/x/run_kernel_stats.csv [--top 15]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    for f in a.csv:
        rows = list(csv.DictReader(open(f)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
        print(f)
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
            name = r["Name"].split("(")[0].replace("void ", "")
            print("  %-60s %6s calls %9.1f us avg %5.1f %%" % (name[:60], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                               100 * float(r["TotalDurationNs"]) / tot))


if __name__ == "__main__":
    main()
