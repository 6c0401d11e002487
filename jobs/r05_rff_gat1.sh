#!/bin/bash
# Round 5: (1) Fourier-feature MMD on the wide form from D > 32: tests + d = 200 timing;
# (2) papers100M dry run (rank 0 of 8, scale 0.5) A/B of the XCD remap in the GAT kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_rff_gat1
mkdir -p $O
( while sleep 20; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "rff or fast or fourier or Fourier" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for spec in "200 400" "64 128" "300 600"; do
  set -- $spec
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --R 32 --n 500 --train 20 --test 10 --fast >> $O/time_fast.jsonl 2> $O/err_$1.log || { echo "d=$1 failed"; tail $O/err_$1.log; exit 1; }
  tail -n 1 $O/time_fast.jsonl | cut -c1-250
done
for v in base gat64 gat512; do
  if [ $v = base ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abv/$v/_hip.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 900 python -u tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --partition locality --scale 0.5 --steps 8 --warmup 2 --order-cache /tmp/order_p05.npy > $O/papers_$v.log 2>&1 || { echo papers $v failed; tail -n 20 $O/papers_$v.log; exit 1; }
  echo $v $(grep '^{' $O/papers_$v.log | cut -c1-260)
done
echo done
