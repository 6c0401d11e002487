"""Summarise a rocprofv3 database (``--kernel-trace`` run, rocpd SQLite output) into
per-kernel totals: calls, total / average time and share.  Writes CSV to stdout.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--top 25]
"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), max(vgpr_count), "
                     "max(accum_vgpr_count), max(lds_size) from kernels group by name "
                     "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "pct", "vgpr", "agpr", "lds_bytes"])
    for r in rows[:a.top]:
        w.writerow([r[0][:160], r[1], round(r[2] / 1e3, 1), round(r[3] / 1e3, 2), round(100 * r[2] / tot, 2),
                    r[4], r[5], r[6]])


if __name__ == "__main__":
    main()
