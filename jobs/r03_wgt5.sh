#!/bin/bash
# lin_bwd_weight2 with gathered first operands (row ids staged in LDS): tests, SAGE layer-0 kernel A/B, SAGE config
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_wgt5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o lin -- python tools/bench_lin.py --reps 5 --rows 60000 200000 > $O/prof.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sage_prof -o run -- python3 -u tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/sage_prof.log 2>&1
find $O -name "*_trace.csv" -size +3M -delete
