#!/bin/bash
# GraphSAGE with one sampler stream (and scratch) per pipeline slot, raw current-stream
# pointers in the launch helpers: the whole GPU suite, the host-time probe and the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_sage_streams
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -u tools/sage_host.py > $O/host.log 2>&1 || { echo host probe failed; tail $O/host.log; exit 1; }
grep '^{' $O/host.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
  tail -n 1 $O/sage_$r.log | cut -c1-220
done
echo done
