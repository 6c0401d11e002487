#!/bin/bash
# Round 6: GraphSAGE sampler and training on disjoint CU sets (CU-masked streams)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_cumask
mkdir -p $O
for r in 1 2; do
for c in 32 0 64 16; do
CGNN_SAGE_SAMPLER_CUS=$c timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_c${c}_$r.log 2>&1 || { echo sage failed; tail $O/sage_c${c}_$r.log; exit 1; }
echo "cus $c run $r: $(grep -o '"value": [0-9.]*' $O/sage_c${c}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_c${c}_$r.log)"
done
done
echo done
