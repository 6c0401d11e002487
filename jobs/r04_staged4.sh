#!/bin/bash
# staged generator kernels: batched input gathers; A/B of W x placement; d = 200 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_staged4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_cgnn_wide_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
for h in 20 100; do
  timeout -k 10 300 python -u tools/ab_staged.py --h $h > $O/ab_h$h.log 2>&1 || { echo "ab h$h failed"; tail $O/ab_h$h.log; exit 1; }
  cat $O/ab_h$h.log | grep -v amdgpu.ids
done
for cfg in "20 256" "100 256"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R $2 --n 500 --h $1 --train 50 --test 20 > $O/d200_h$1_r$2.log 2>&1 || { echo "bench h$1 r$2 failed"; tail $O/d200_h$1_r$2.log; exit 1; }
  tail -n 1 $O/d200_h$1_r$2.log
done
echo done
