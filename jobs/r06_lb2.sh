#!/bin/bash
# Round 6: look-back sampler (in-tree, 4 launches per level) vs HEAD (7 per level), interleaved, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_lb2
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/head/_hip.cpython-310-x86_64-linux-gnu.so
for r in 1 2 3; do
for v in new old; do
L=""; [ $v = old ] && L=$OLD
CGNN_HIP_LIB=$L timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "sage $v $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
for v in new old; do
L=""; [ $v = old ] && L=$OLD
CGNN_HIP_LIB=$L timeout -k 10 300 python -u tools/sage_sampler_only.py > $O/so_${v}.log 2>&1 || { echo so failed; tail $O/so_${v}.log; exit 1; }
echo "sampler-only $v: $(grep '^{' $O/so_${v}.log)"
done
echo done
