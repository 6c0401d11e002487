#!/bin/bash
# Round 6: GraphSAGE input features at a 256-B row pitch (whole 128-B lines) vs 208 B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_xpad
mkdir -p $O
for r in 1 2; do
for v in 128 0; do
CGNN_SAGE_XPAD=$v timeout -k 10 300 python -u tools/sage_train_only.py --steps 192 > $O/to_${v}_$r.log 2>&1 || { echo failed; tail $O/to_${v}_$r.log; exit 1; }
echo "pad $v train-only $r: $(grep -o '"train_only_us_per_step": [0-9.]*' $O/to_${v}_$r.log)"
CGNN_SAGE_XPAD=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "pad $v sage $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
echo done
