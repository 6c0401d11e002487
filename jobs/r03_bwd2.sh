#!/bin/bash
# Round 3: the rows x hidden fused dense backward (gcn_fused_bwd2_kernel) -- its
# numerics tests, an A/B against the round-2 form, a kernel trace of the headline
# epoch, then the whole GPU suite, smoke and the SAGE copy trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_bwd2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "fused_backward or benched_config or hipgraph or train_row or steps_match or fused_dense" > $O/pytest_bwd.log 2>&1 \
    || { echo "bwd tests failed"; grep -E "FAILED|Error|assert" $O/pytest_bwd.log | head -20; tail -n 30 $O/pytest_bwd.log; exit 1; }
tail -n 1 $O/pytest_bwd.log
for v in 0 1 0 1; do
  CGNN_FUSED_BWD_V1=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_v1_$v.log 2>&1 || { echo bench failed; tail $O/bench_v1_$v.log; exit 1; }
  echo "v1=$v $(tail -n 1 $O/bench_v1_$v.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_bwd2/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:14]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
find $O -name "*_trace.csv" -delete
bash jobs/r03_full.sh && bash jobs/r03_sage.sh
