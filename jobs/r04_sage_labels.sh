#!/bin/bash
# GraphSAGE with the epoch's labels gathered once: sampler / SAGE GPU tests and the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_sage_labels
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py tests/test_gnn_gpu.py -k "sage or sampler or pipelined" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
  tail -n 1 $O/sage_$r.log | cut -c1-160
done
echo done
