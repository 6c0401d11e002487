#!/bin/bash
# lin_fwd / lin_bwd_data at K = 256: 16-wave blocks (in-tree) vs 8-wave blocks with the
# branch-free loader and a 256-VGPR budget (abtmp/bwd8: lin_bwd_data only; abtmp/both8: both)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_waves
mkdir -p $O
for v in new bwd8 both8; do
  lib=""
  [ $v != new ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail $O/tests_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lin_$v -o run -- python3 tools/bench_lin.py --reps 5 --rows 60000 200000 > $O/lin_$v.log 2>&1 || { echo "lin $v failed"; tail $O/lin_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$v.log 2>&1 || { echo "arxiv $v failed"; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$v.log 2>&1 || { echo "sage $v failed"; exit 1; }
  echo "$v $(tail -n 1 $O/tests_$v.log)"; tail -n 1 $O/arxiv_$v.log | cut -c90-170; tail -n 1 $O/sage_$v.log | cut -c100-180
done
find $O -name "*_trace.csv" -size +3M -delete
