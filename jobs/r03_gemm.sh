#!/bin/bash
# Round 3: tiled lin_gemm kernel (wide-K dense layer) -- linear-layer GPU tests, Reddit
# inference A/B (CGNN_LIN_GEMM 1 / 0), kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_gemm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_linear_gpu.py tests/test_gnn_gpu.py -k "lin or inference or deep" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
echo "$(tail -n 1 $O/pytest.log)"
for v in 1 0; do
  CGNN_LIN_GEMM=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_$v.log 2>&1 || { echo bench failed; tail $O/reddit_$v.log; exit 1; }
  echo "gemm=$v $(tail -n 1 $O/reddit_$v.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_gemm/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find $O -name "*_trace.csv" -delete
echo done
