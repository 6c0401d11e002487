#!/bin/bash
# lin_fwd / lin_bwd_data A/B on the arxiv config: nontemporal output stores, 4-wave
# blocks for K = 256, 8-wave prefetching blocks for K = 128
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin2
mkdir -p $O
for v in base nt w4 f8w8 ntf8; do
  lib=""
  [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/arxiv_$v -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 --steps 50 > $O/arxiv_prof_$v.log 2>&1 || { echo "arxiv prof $v failed"; tail $O/arxiv_prof_$v.log; exit 1; }
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$v.log 2>&1 || { echo "arxiv $v failed"; tail $O/arxiv_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/arxiv_$v.log | cut -c90-160)"
done
find $O -name "*_trace.csv" -delete
