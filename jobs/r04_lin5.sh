#!/bin/bash
# weight-stationary lin_fwd / lin_bwd_data (in-tree) vs the slab kernels (nows)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -v PASSED $O/tests.log | tail -n 40; exit 1; }
tail -n 1 $O/tests.log
for v in base nows; do
  lib=""
  [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail $O/kt_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/kt_$v.log)"
  CGNN_HIP_LIB=$lib timeout -k 10 200 python3 tools/bench_lin.py --reps 10 --rows 200000 > $O/sagelin_$v.log 2>&1 || { echo "sagelin $v failed"; tail $O/sagelin_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/sagelin_$v.log)"
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$v.log 2>&1 || { echo "arxiv $v failed"; tail $O/arxiv_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/arxiv_$v.log | cut -c90-160)"
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$v.log 2>&1 || { echo "sage $v failed"; tail $O/sage_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/sage_$v.log | cut -c90-170)"
done
find $O -name "*_trace.csv" -delete
