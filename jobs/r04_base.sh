#!/bin/bash
# Round 4 baseline: the GPU suite, smoke, headline bench, kernel trace of the headline epoch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_base
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -n 30 $O/pytest_gpu.log; exit 1; }
echo "$(tail -n 1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-200
B="python3 -u bench.py --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $B > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04_base/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:14]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
find $O -name "*_trace.csv" -delete
echo done
