#!/bin/bash
# 4-rank rehearsal on one GPU (gloo), backward all-gather overlap off / on
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/rehearse_ab
mkdir -p $O
for ov in 0 1; do
  CGNN_BWD_OVERLAP=$ov timeout -k 10 240 python -u bench.py --gpus 4 --shared-gpu --steps 3 --warmup 1 --scale 0.25 > $O/r4_ov$ov.log 2>&1 &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 15; kill -0 $pid 2>/dev/null && echo "overlap=$ov running"; done
  wait $pid; rc=$?
  echo "overlap=$ov rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4_ov$ov.log) $(grep -o '"setup_s": [0-9.]*' $O/r4_ov$ov.log)"
  [ $rc -eq 0 ] || exit 1
done
