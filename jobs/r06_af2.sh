#!/bin/bash
# Round 6: A/B of the Adam step fold + SAGE summed losses (new) against the separate launches (old), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_af2
mkdir -p $O
for r in 1 2 3; do
for v in new old; do
E="CGNN_ADAM_FOLD=1 CGNN_SAGE_SUMMED=1"; [ $v = old ] && E="CGNN_ADAM_FOLD=0 CGNN_SAGE_SUMMED=0"
env $E timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "sage $v $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
echo done
