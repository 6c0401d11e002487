#!/bin/bash
# weight-gradient chunk count A/B with the final lin_bwd_weight2 (env knobs only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_chunks
mkdir -p $O
for v in 1 2; do
  CGNN_WGT2_CHUNK_DIV=$v timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wgrad_div$v.json 2> $O/wgrad_div$v.err || { echo "wgrad $v failed"; exit 1; }
  CGNN_WGT2_CHUNK_DIV=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_div$v.log 2>&1 || { echo "sage $v failed"; exit 1; }
  CGNN_WGT2_CHUNK_DIV=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_div$v.log 2>&1 || { echo "arxiv $v failed"; exit 1; }
done
for v in 1 2; do cat $O/wgrad_div$v.json; tail -n 1 $O/sage_div$v.log | cut -c100-180; tail -n 1 $O/arxiv_div$v.log | cut -c90-170; done
