#!/bin/bash
# Round 6: GraphSAGE epoch keeps per-batch loss sums (no per-batch division launch) vs dividing per batch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_summed
mkdir -p $O
for r in 1 2 3; do
for v in 1 0; do
CGNN_SAGE_SUMMED=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "summed $v run $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
echo done
