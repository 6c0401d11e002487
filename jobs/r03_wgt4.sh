#!/bin/bash
# lin_bwd_weight2 with unconditional (clamped) loads, validity / mask applied at staging
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_wgt4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py tests/test_gnn_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_new.json 2> $O/wgrad_new.err &&
CGNN_WGT_V1=1 timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_v1.json 2> $O/wgrad_v1.err &&
CGNN_WGT2_MIN_TILES=4 timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_m4.json 2> $O/wgrad_m4.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o wg -- python tools/bench_wgrad.py --reps 5 > $O/prof.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_new.log 2>&1 &&
CGNN_WGT_V1=1 timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_v1.log 2>&1
