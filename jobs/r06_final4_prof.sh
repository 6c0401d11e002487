#!/bin/bash
# Round 6: kernel traces of the committed tree (headline epoch, GraphSAGE batch)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_final4/prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gcn -o run -- python3 bench.py --steps 10 --warmup 3 > $O/gcn_prof.log 2>&1 || { echo prof failed; tail $O/gcn_prof.log; exit 1; }
python3 tools/epoch_trace.py $O/gcn/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sage -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/sage_prof.log 2>&1 || { echo prof failed; tail $O/sage_prof.log; exit 1; }
python3 tools/sage_trace.py $O/sage > $O/sage_trace.txt 2>&1 || true
head -8 $O/sage_trace.txt
cp $O/gcn/run_kernel_stats.csv $O/gcn_kernel_stats.csv; cp $O/sage/run_kernel_stats.csv $O/sage_kernel_stats.csv
rm -rf $O/gcn $O/sage
echo done
