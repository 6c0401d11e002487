#!/bin/bash
# weight-stationary kernels reading the fp32 master weights directly (no image kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py tests/test_gnn_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt.log 2>&1 || { echo "kt failed"; tail $O/kt.log; exit 1; }
grep '^{' $O/kt.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/arxiv_kt -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 --steps 50 > $O/arxiv_kt.log 2>&1 || { echo "arxiv kt failed"; tail $O/arxiv_kt.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$i.log 2>&1 || { echo "arxiv failed"; tail $O/arxiv_$i.log; exit 1; }
  tail -n 1 $O/arxiv_$i.log | cut -c90-160
done
find $O -name "*_trace.csv" -delete
