#!/bin/bash
# weight-stationary kernels after the wait-count fixes (staged row ids / scales, unconditional ring loads): ring 5 vs 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in base ring3; do
  lib=""
  [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail $O/kt_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/kt_$v.log)"
done
timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo "arxiv failed"; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log | cut -c90-160
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo "sage failed"; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c90-170
find $O -name "*_trace.csv" -delete
