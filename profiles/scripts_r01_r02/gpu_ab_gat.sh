#!/bin/bash
# A/B of GAT aggregation-kernel variants (abtmp/<name>/_hip*.so) against the in-tree build
# on the products-shape fused GAT epoch; GAT GPU tests on the in-tree build first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_gat
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -k gat -x -q --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in intree "$@" intree "$@"; do
  if [ $v = intree ]; then lib=""; else lib=$(ls abtmp/$v/_hip*.so); fi
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_epoch": [0-9.]*' $O/$v.log)"
done
