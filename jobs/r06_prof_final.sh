#!/bin/bash
# Round 6: closing kernel trace of the headline epoch and of a GraphSAGE epoch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_prof_final
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gcn -o run -- python3 bench.py --steps 10 --warmup 3 > $O/gcn.log 2>&1 || { echo prof failed; tail $O/gcn.log; exit 1; }
python3 tools/epoch_trace.py $O/gcn/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
find $O/gcn -name "*kernel_trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sage -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/sage.log 2>&1 || { echo prof failed; tail $O/sage.log; exit 1; }
python3 tools/sage_trace.py $O/sage > $O/sage_trace.txt 2>&1 || true
head -6 $O/sage_trace.txt
find $O/sage -name "*kernel_trace.csv" -delete
echo done
