#!/bin/bash
# Round 6: GraphSAGE per-batch stream view (kernel trace of one epoch)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sagetr
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 tools/sage_trace.py $O/trace > $O/sage_trace.txt 2>&1 || true
cat $O/sage_trace.txt | head -60
echo done
