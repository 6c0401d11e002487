#!/bin/bash
# Round 5: kernel family by variable count (per-sample up to 32 variables): the CGNN GPU
# tests, and the family timings again through the default ("auto") path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_family2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_cgnn_kernels_gpu.py tests/test_cgnn_wide_gpu.py tests/test_examples_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for spec in "22 30 0" "40 80 0" "64 128 0" "100 200 0"; do
  set -- $spec
  timeout -k 10 200 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --conf $3 --R 256 --n 500 --h 20 --train 100 --test 50 >> $O/family.jsonl 2> $O/err.log || { echo "d=$1 failed"; tail $O/err.log; exit 1; }
  tail -n 1 $O/family.jsonl | cut -c1-260
done
echo done
