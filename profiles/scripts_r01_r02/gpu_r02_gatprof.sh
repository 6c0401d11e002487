#!/bin/bash
# Kernel-time profile of the fused GAT epoch (products shape, reorder pass) and the
# 3-layer SAGE epoch; plus the GCN headline after the small-kernel trim.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gatprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gat -o run -- python -u tools/bench_gat.py --steps 5 --warmup 1 > $O/gat.log 2>&1 || { echo gat failed; tail $O/gat.log; exit 1; }
grep -h '"value"\|ms' $O/gat.log | tail -2
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $O/bench.log
echo done
