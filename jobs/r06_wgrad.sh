#!/bin/bash
# Round 6: GraphSAGE weight-gradient split-K chunk count (device_cus / slabs / DIV) A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_wgrad_mq
mkdir -p $O
for r in 1 2; do
for v in 4 6 8; do
CGNN_WGRAD_MQ=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "mq $v run $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
echo done
