#!/bin/bash
# lin_fwd / lin_bwd_data loader A/B: in-tree (branch-free X loader at KS >= 16, branch-free
# gradient loader in lin_bwd_data except the 16-wave KN = 16 variant) vs the previous
# branchy loaders (abtmp/lin_old) vs branch-free X loader from KS = 8 (abtmp/lin_ks8)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_linsel
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in new old ks8; do
  lib=""
  [ $v != new ] && lib=$PWD/abtmp/lin_$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lin_$v -o run -- python3 tools/bench_lin.py --reps 5 --rows 60000 200000 > $O/lin_$v.log 2>&1 || { echo "lin $v failed"; tail $O/lin_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$v.log 2>&1 || { echo "sage $v failed"; tail $O/sage_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_$v.log 2>&1 || { echo "gat $v failed"; tail $O/gat_$v.log; exit 1; }
  tail -n 1 $O/sage_$v.log | cut -c1-200
done
find $O -name "*_trace.csv" -size +3M -delete
echo done
