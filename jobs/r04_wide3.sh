#!/bin/bash
# d > 256 on the GPU (grouped matrix-core MMD) + the time-boxed orient_directed_graph run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_wide3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_cgnn_wide_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for d in 300 512; do
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d $d --edges $((2 * d)) --R 256 --n 500 --h 20 --train 30 --test 10 > $O/d${d}_h20_r256.log 2>&1 || { echo "bench d$d failed"; tail $O/d${d}_h20_r256.log; exit 1; }
  tail -n 1 $O/d${d}_h20_r256.log
done
timeout -k 10 480 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail -20 $O/orient.log; exit 1; }
tail -n 1 $O/orient.log
