#!/bin/bash
# lin_fwd KS = 8 (GAT projection, K = 100): 16-wave (in-tree) vs 8-wave blocks (abtmp/fwd8w)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_fwd8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests_new.log 2>&1 || { echo tests failed; tail -30 $O/tests_new.log; exit 1; }
tail -n 1 $O/tests_new.log
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new.log 2>&1 || { echo sage failed; exit 1; }
tail -n 1 $O/sage_new.log | cut -c100-180
for v in new fwd8w new2 fwd8w2; do
  lib=""
  case $v in fwd8w*) lib=$PWD/abtmp/fwd8w/_hip.cpython-310-x86_64-linux-gnu.so;; esac
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_$v.log 2>&1 || { echo "gat $v failed"; tail $O/gat_$v.log; exit 1; }
  echo "$v $(grep -h ms_per_epoch $O/gat_$v.log | cut -c95-170)"
done
CGNN_HIP_LIB=$PWD/abtmp/fwd8w/_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests_fwd8w.log 2>&1 || { echo tests failed; tail $O/tests_fwd8w.log; exit 1; }
tail -n 1 $O/tests_fwd8w.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_new -o run -- python3 -u tools/bench_gat.py --steps 3 --warmup 1 > $O/t_new.log 2>&1 || exit 1
CGNN_HIP_LIB=$PWD/abtmp/fwd8w/_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_fwd8w -o run -- python3 -u tools/bench_gat.py --steps 3 --warmup 1 > $O/t_fwd8w.log 2>&1 || exit 1
find $O -name "*_trace.csv" -size +3M -delete
