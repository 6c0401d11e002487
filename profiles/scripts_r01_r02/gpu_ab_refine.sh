#!/bin/bash
# A/B of the reorder pass's median-smoothing refinement (CGNN_REORDER_REFINE rounds)
# on the headline GCN epoch.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_refine
mkdir -p $O
for r in ${@:-0 4 8}; do
  CGNN_REORDER_REFINE=$r timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/bench_refine$r.log 2>&1 || exit 1
  echo "refine=$r $(grep -o '"value": [0-9.]*' $O/bench_refine$r.log) $(grep -o '"trainer_setup_s": [0-9.]*' $O/bench_refine$r.log)"
done
