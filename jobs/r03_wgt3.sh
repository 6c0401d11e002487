#!/bin/bash
# lin_bwd_weight2 with a two-deep register ring; lin_fwd / lin_bwd_data grid A/B (tiles per block)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_wgt3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_new.json 2> $O/wgrad_new.err &&
CGNN_WGT_V1=1 timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_v1.json 2> $O/wgrad_v1.err &&
timeout -k 10 200 python -u tools/bench_lin.py > $O/lin.json 2> $O/lin.err &&
CGNN_LIN_TILES_PER_BLOCK=4 timeout -k 10 200 python -u tools/bench_lin.py > $O/lin_t4.json 2> $O/lin_t4.err &&
CGNN_WGT2_MIN_TILES=2 timeout -k 10 200 python -u tools/bench_lin.py > $O/lin_m2.json 2> $O/lin_m2.err &&
CGNN_WGT2_MIN_TILES=4 timeout -k 10 200 python -u tools/bench_lin.py > $O/lin_m4.json 2> $O/lin_m4.err &&
CGNN_LIN_TILES_PER_BLOCK=1 timeout -k 10 200 python -u tools/bench_lin.py > $O/lin_t1.json 2> $O/lin_t1.err &&
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new.log 2>&1 &&
CGNN_LIN_TILES_PER_BLOCK=4 timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_t4.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_new.log 2>&1 &&
CGNN_WGT_V1=1 timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_v1.log 2>&1
