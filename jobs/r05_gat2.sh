#!/bin/bash
# Round 5: GAT kernels on the chunk-interleaved XCD remap: GAT GPU tests, then the full
# papers100M rank-0-of-8 dry run (the 75 ms epoch of round 4) with a kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_gat2
mkdir -p $O
( while sleep 20; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_gat_fused_gpu.py -x -q --timeout 300 --timeout-method thread -k "gat or GAT" > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 700 python3 tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --partition locality --steps 10 --warmup 2 --order-cache /tmp/order_full.npy > $O/papers_dry.log 2>&1 || { echo papers failed; tail -n 20 $O/papers_dry.log; exit 1; }
grep '^{' $O/papers_dry.log | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --partition locality --steps 5 --warmup 2 --order-cache /tmp/order_full.npy > $O/papers_dry_prof.log 2>&1 || { echo papers prof failed; tail -n 20 $O/papers_dry_prof.log; exit 1; }
grep '^{' $O/papers_dry_prof.log | cut -c1-200
echo done
