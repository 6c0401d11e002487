#!/bin/bash
# Multi-rank HIP path rehearsed on one GPU (gloo collectives, every rank on cuda:0):
# 1, 2 and 4 ranks of the headline GCN must report the same training loss.  A heartbeat
# line every 20 s while a run is in progress (4 ranks share one box's CPUs for setup).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/rehearse
mkdir -p $O
SCALE=${SCALE:-1.0}
for w in 1 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $w --shared-gpu --steps 5 --warmup 2 --scale $SCALE > $O/rehearse$w.log 2>&1 &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "ranks=$w running"; done
  wait $pid || { echo "rehearsal $w failed"; tail -20 $O/rehearse$w.log; exit 1; }
  echo "ranks=$w $(grep -o '"train_loss": [0-9.]*' $O/rehearse$w.log) $(grep -o '"val_acc": [0-9.]*' $O/rehearse$w.log) $(grep -o '"ms_per_step": [0-9.]*' $O/rehearse$w.log)"
done
