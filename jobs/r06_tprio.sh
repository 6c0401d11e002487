#!/bin/bash
# Round 6: GraphSAGE training stream at high priority (-1) vs normal (0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_tprio
mkdir -p $O
for r in 1 2 3; do
for c in -1 0; do
CGNN_SAGE_TRAIN_PRIO=$c timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_p${c}_$r.log 2>&1 || { echo sage failed; tail $O/sage_p${c}_$r.log; exit 1; }
echo "prio $c run $r: $(grep -o '"value": [0-9.]*' $O/sage_p${c}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_p${c}_$r.log)"
done
done
echo done
