#!/bin/bash
# 16-byte-load weight-gradient reduce (lin_reduce4_kernel): linear-layer / GNN GPU tests,
# arxiv kernel trace, arxiv / SAGE benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_reduce
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_linear_gpu.py tests/test_gnn_gpu.py tests/test_sampler_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 --steps 20 --warmup 5 > $O/arxiv_kt.log 2>&1 || { echo arxiv kt failed; tail $O/arxiv_kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -n 1)
cp $f $O/arxiv_kernel_stats.csv
python3 tools/kstats.py $O/arxiv_kernel_stats.csv --top 12
find $O -name "*_trace.csv" -delete
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$r.log 2>&1 || { echo arxiv failed; tail $O/arxiv_$r.log; exit 1; }
  tail -n 1 $O/arxiv_$r.log | cut -c1-160
done
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c1-160
echo done
