#!/bin/bash
# Round 4: forward with per-wave LDS-DMA row staging (8 waves / CU) -- tests, A/B vs the
# previous commit's kernels, headline bench, one-epoch trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_fwd2
mkdir -p $O
# timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_gnn.log 2>&1 \
#    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gnn.log | head -20; tail -n 30 $O/pytest_gnn.log; exit 1; }
# echo "$(tail -n 1 $O/pytest_gnn.log)"
for round in 1 2; do
  for v in default prev fwd_dma_unroll fwd_dma_sp; do
    if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$(ls $PWD/abtmp/$v/_hip*.so); fi
    timeout -k 10 120 python -u tools/ab_dense.py --iters 30 >> $O/ab.log 2>&1 || { echo "ab $v failed"; tail $O/ab.log; exit 1; }
  done
done
unset CGNN_HIP_LIB
grep '{' $O/ab.log | cut -c1-150
# timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
# tail -n 1 $O/bench.log | cut -c1-160
B="python3 -u bench.py --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- $B > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $(find $O/prof -name "*kernel_trace.csv" | head -1) 4 > $O/epoch.txt
cat $O/epoch.txt
find $O -name "*_trace.csv" -delete
echo done
