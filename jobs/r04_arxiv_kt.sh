#!/bin/bash
# layer-1 SpMM column-slab A/B, arxiv-gcn3 per-kernel breakdown (kernel trace of a short run) and the SAGE run with the
# input layer's global source ids taken from the sampler's picks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_arxiv_kt
mkdir -p $O
timeout -k 10 400 python -u tools/ab_spmm_slab.py --rounds 3 > $O/ab_slab.log 2>&1 || { echo slab ab failed; tail $O/ab_slab.log; exit 1; }
cat $O/ab_slab.log | grep '^{'
for r in 1 2; do
  for sl in 0; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_slab${sl}_$r.log 2>&1 || { echo bench failed; tail $O/bench_slab${sl}_$r.log; exit 1; }
    echo "slab $sl: $(grep '^{' $O/bench_slab${sl}_$r.log | cut -c1-150)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 --steps 20 --warmup 5 > $O/arxiv_kt.log 2>&1 || { echo arxiv kt failed; tail $O/arxiv_kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -n 1)
cp $f $O/arxiv_kernel_stats.csv
python3 tools/kstats.py $O/arxiv_kernel_stats.csv --top 20
find $O -name "*_trace.csv" -delete
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c1-200
echo done
