#!/bin/bash
# lin_fwd / lin_bwd_data packed epilogue + next-tile prefetch: tests, kernel trace at the
# SAGE layer-0 shapes and on the arxiv / SAGE configs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py tests/test_gnn_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lin -o run -- python3 tools/bench_lin.py --reps 5 --rows 60000 200000 > $O/lin.log 2>&1 || { echo "lin failed"; tail $O/lin.log; exit 1; }
grep '^{' $O/lin.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/arxiv -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_prof.log 2>&1 || { echo "arxiv prof failed"; tail $O/arxiv_prof.log; exit 1; }
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo "arxiv failed"; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log | cut -c1-400
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo "sage failed"; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c1-400
find $O -name "*_trace.csv" -size +3M -delete
