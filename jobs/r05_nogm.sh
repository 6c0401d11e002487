#!/bin/bash
# Round 5: staged CGNN backward without the Gm LDS rows (dW2 from the MFMA registers, 14-float mg rows) against
# the committed 12-unit-chunk build (default lib)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_nogm
mkdir -p $O
V=$PWD/abv/nogm/_hip.cpython-310-x86_64-linux-gnu.so
CGNN_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "staged or wide" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for e in 736 400; do
for v in default nogm default nogm; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$V; fi
  timeout -k 10 300 python -u tools/ab_staged.py --d 200 --edges $e --R 256 --n 500 --h 20 --only bwd:4:2 > $O/ab_${v}_$e.log 2>&1 || { echo ab $v failed; tail $O/ab_${v}_$e.log; exit 1; }
  echo $v $e $(grep bwd $O/ab_${v}_$e.log)
done
done
for v in default nogm; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$V; fi
  for e in 736 400; do
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges $e --R 256 --n 500 --h 20 > $O/batch_${v}_$e.log 2>&1 || { echo batch $v failed; tail $O/batch_${v}_$e.log; exit 1; }
  echo $v $e $(grep '^{' $O/batch_${v}_$e.log | cut -c1-300)
  done
done
echo done
