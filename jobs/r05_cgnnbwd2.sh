#!/bin/bash
# Round 5: staged CGNN backward with the dL/dparent partials in registers (4 blocks per CU
# instead of 3 at d = 200) and Gm on v_mfma_f32_16x16x4_f32; tests, A/B, GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_cgnnbwd2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "staged or wide" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in hz16 new; do
  if [ $v = new ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abv/$v/_hip.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 300 python -u tools/ab_staged.py --d 200 --edges 400 --R 256 --n 500 --h 20 --only bwd:4:2 > $O/ab_$v.log 2>&1 || { echo ab $v failed; tail $O/ab_$v.log; exit 1; }
  echo $v $(grep bwd $O/ab_$v.log)
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 256 --n 500 --h 20 > $O/batch_$v.log 2>&1 || { echo batch $v failed; tail $O/batch_$v.log; exit 1; }
  echo $v $(grep '^{' $O/batch_$v.log | cut -c1-300)
done

timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_suite.log | head -20
tail -n 2 $O/gpu_suite.log
exit $rc
