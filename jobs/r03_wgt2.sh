#!/bin/bash
# lin_bwd_weight2 with raw prefetch: numerics, A/B (chunk count), SAGE layer-0 dense kernels, SAGE / GAT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_wgt2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_new.json 2> $O/wgrad_new.err &&
CGNN_WGT2_CHUNK_DIV=2 timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_div2.json 2> $O/wgrad_div2.err &&
timeout -k 10 200 python -u tools/bench_lin.py > $O/lin.json 2> $O/lin.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o lin -- python tools/bench_lin.py --reps 5 --rows 60000 > $O/prof.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_new.log 2>&1 &&
CGNN_WGT_V1=1 timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_v1.log 2>&1
