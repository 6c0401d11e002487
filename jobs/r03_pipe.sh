#!/bin/bash
# Round 3: fused backward bit-mode draw placement A/B (CGNN_BWD_PIPE 0 / 1 / 2), GNN tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_pipe
mkdir -p $O
for v in 0 1 2; do
  CGNN_BWD_PIPE=$v timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or benched or hipgraph or train_row" > $O/pytest_$v.log 2>&1 \
    || { echo "tests failed $v"; grep -E "FAILED|Error|assert" $O/pytest_$v.log | head -20; tail -n 30 $O/pytest_$v.log; exit 1; }
  echo "pipe=$v $(tail -n 1 $O/pytest_$v.log)"
done
for v in 0 1 2 0 1 2; do
  CGNN_BWD_PIPE=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$v.log 2>&1 || { echo bench failed; tail $O/bench_$v.log; exit 1; }
  echo "pipe=$v $(tail -n 1 $O/bench_$v.log | cut -c1-150)"
done
for v in 0 1 2; do
  CGNN_BWD_PIPE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/prof$v.log 2>&1 || { echo prof failed; tail $O/prof$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in "012":
    f = glob.glob("gpurun_out/r03_pipe/prof%s/**/*kernel_stats.csv" % v, recursive=True)
    for r in list(csv.DictReader(open(f[0]))):
        if "gcn_" in r["Name"]:
            print(v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us min", round(float(r["MinNs"]) / 1e3, 1))
PY
find $O -name "*_trace.csv" -delete
echo done
