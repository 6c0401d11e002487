#!/bin/bash
# Round 5: weight-gradient reduce over 32 lane groups (was 8): linear / SAGE tests, then
# products-sage3 x2 and arxiv-gcn3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_reduce1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_linear_gpu.py tests/test_sampler_gpu.py tests/test_gnn_gpu.py -x -q --timeout 300 --timeout-method thread -k "lin or sage or sampler or arxiv or gcn3" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
tail -n 1 $O/sage_$r.log | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo arxiv failed; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo done
