#!/bin/bash
# Round 4: A/B of forward forms: LDS-DMA staging (8 waves) plain / hidden loop unrolled /
# software-pipelined, against the committed 16-wave form (prev)
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
echo done
