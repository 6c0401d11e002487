#!/bin/bash
# arxiv-gcn3 kernel trace (where the 0.85 ms epoch goes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_arxiv_prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u tools/bench_gnn_configs.py --config arxiv-gcn3 --steps 20 --warmup 3 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 - <<'PY' > $O/summary.txt
import csv, glob
f = glob.glob("gpurun_out/r03_arxiv_prof/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
T = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", round(T / 1e6, 2))
for r in rows[:25]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(100 * float(r["TotalDurationNs"]) / T, 1))
PY
cat $O/summary.txt
find $O -name "*_trace.csv" -size +3M -delete
