#!/bin/bash
# Round 3: spmm_ce long-row threshold A/B (CGNN_CE_LONG = 0 disables), kernel traces.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ce2
mkdir -p $O
for v in 0 128 256 512; do
  CGNN_CE_LONG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof$v.log 2>&1 || { echo prof failed; tail $O/prof$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in ("0", "128", "256", "512"):
    f = glob.glob("gpurun_out/r03_ce2/prof%s/**/*kernel_stats.csv" % v, recursive=True)
    for r in list(csv.DictReader(open(f[0]))):
        if "spmm_ce" in r["Name"]:
            print(v, r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us min", round(float(r["MinNs"]) / 1e3, 1))
PY
find $O -name "*_trace.csv" -delete
echo done
