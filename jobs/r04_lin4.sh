#!/bin/bash
# lin_fwd / lin_bwd_data output staging through LDS (in-tree) vs direct 8-B stores (notst);
# tests first; arxiv-shape kernel trace + write-request PMC; arxiv / SAGE configs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in base notst; do
  lib=""
  [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail $O/kt_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/kt_$v.log)"
  CGNN_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/pmc_$v -o run -- python3 tools/bench_lin.py --shape arxiv --reps 2 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail $O/pmc_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$v.log 2>&1 || { echo "arxiv $v failed"; tail $O/arxiv_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/arxiv_$v.log | cut -c90-160)"
  CGNN_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_$v -o run -- python3 tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_$v.log 2>&1 || { echo "reddit $v failed"; tail $O/reddit_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/reddit_$v.log | cut -c90-170)"
done
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo "sage failed"; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c90-170
find $O -name "*_trace.csv" -delete
