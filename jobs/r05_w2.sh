#!/bin/bash
# Round 5: the staged backward planned at 2 waves per block: staged / wide GPU tests, the
# d = 200 train step at 400 and 736 edges, and the reference-settings orientation run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_w2
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for e in 400 736; do
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges $e --R 256 --n 500 --h 20 > $O/batch_$e.log 2>&1 || { echo batch failed; tail $O/batch_$e.log; exit 1; }
  echo $e $(grep '^{' $O/batch_$e.log | cut -c1-300)
done
timeout -k 10 400 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 1 $O/orient.log | cut -c1-400
echo done
