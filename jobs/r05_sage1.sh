#!/bin/bash
# Round 5: where the SAGE mini-batch time goes -- API trace (what the copyBuffer calls
# are), kernel trace; plus the CGNN wide-width timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_sage1
mkdir -p $O
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c1-300
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
ls $O/trace
bash jobs/r05_ell1.sh && bash jobs/r05_cgnn_time.sh
echo done
