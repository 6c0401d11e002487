#!/bin/bash
# Round 3: fused dense backward, hidden blocks per wave (TB) A/B: tests for both forms,
# bench epochs for TB 2 / 1 / the round-2 kernel, kernel trace at the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_tb
mkdir -p $O
for tb in 2 1; do
  CGNN_FUSED_BWD_TB=$tb timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused_backward or benched_config or hipgraph or train_row or steps_match" > $O/pytest_tb$tb.log 2>&1 \
    || { echo "tests failed tb=$tb"; grep -E "FAILED|Error|assert" $O/pytest_tb$tb.log | head -20; tail -n 30 $O/pytest_tb$tb.log; exit 1; }
  echo "tb=$tb $(tail -n 1 $O/pytest_tb$tb.log)"
done
for v in tb2 tb1 v1 tb2 tb1 v1; do
  case $v in tb2) E="CGNN_FUSED_BWD_TB=2";; tb1) E="CGNN_FUSED_BWD_TB=1";; v1) E="CGNN_FUSED_BWD_V1=1";; esac
  env $E timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$v.log 2>&1 || { echo bench failed; tail $O/bench_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/bench_$v.log | cut -c1-180)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_tb/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
find $O -name "*_trace.csv" -delete
echo done
