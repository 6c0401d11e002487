#!/bin/bash
# Round 5: staged CGNN backward capped at 96 VGPRs (5 waves per SIMD where LDS allows) against
# the committed build: backward alone at 400 / 736 edges, and 60-second slices of the
# reference-settings orientation run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_w5
mkdir -p $O
V=$PWD/abv/w5/_hip.cpython-310-x86_64-linux-gnu.so
CGNN_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "staged or wide" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for e in 400 736; do
for v in default w5; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$V; fi
  timeout -k 10 300 python -u tools/ab_staged.py --d 200 --edges $e --R 256 --n 500 --h 20 --only bwd:4:2 > $O/ab_${v}_$e.log 2>&1 || { echo ab $v failed; tail $O/ab_${v}_$e.log; exit 1; }
  echo $v $e $(grep bwd $O/ab_${v}_$e.log)
done
done
for v in default w5; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$V; fi
  timeout -k 10 200 python -u tools/time_orient.py --seconds 60 > $O/orient_$v.log 2>&1 || { echo orient $v failed; tail $O/orient_$v.log; exit 1; }
  echo $v $(tail -n 1 $O/orient_$v.log | cut -c1-400)
done
echo done
