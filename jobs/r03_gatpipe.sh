#!/bin/bash
# Round 3: software-pipelined GAT gather kernels A/B (CGNN_GAT_PIPE 0 / 1 / 2): GAT GPU
# tests per variant, products epoch, kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_gatpipe
mkdir -p $O
for v in 1 2; do
  CGNN_GAT_PIPE=$v timeout -k 10 300 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -k "gat" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 \
    || { echo "tests failed $v"; grep -E "FAILED|Error|assert" $O/pytest_$v.log | head -20; tail -n 30 $O/pytest_$v.log; exit 1; }
  echo "pipe=$v $(tail -n 1 $O/pytest_$v.log)"
done
for v in 0 1 2; do
  CGNN_GAT_PIPE=$v timeout -k 10 300 python -u tools/bench_gat.py --steps 8 --warmup 2 > $O/gat_$v.log 2>&1 || { echo bench failed; tail $O/gat_$v.log; exit 1; }
  echo "pipe=$v $(tail -n 1 $O/gat_$v.log | cut -c1-200)"
done
for v in 0 2; do
  CGNN_GAT_PIPE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/prof$v.log 2>&1 || { echo prof failed; tail $O/prof$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in "02":
    f = glob.glob("gpurun_out/r03_gatpipe/prof%s/**/*kernel_stats.csv" % v, recursive=True)
    for r in list(csv.DictReader(open(f[0]))):
        if "gat_" in r["Name"]:
            print(v, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find $O -name "*_trace.csv" -delete
echo done
