#!/bin/bash
# full-scale 4-rank rehearsal on one GPU (gloo), with periodic stack dumps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/rehearse4
mkdir -p $O
CGNN_TRACEBACK_AFTER=90 timeout -k 10 420 python -u bench.py --gpus 4 --shared-gpu --steps 5 --warmup 2 > $O/r4.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "running $(wc -l < $O/r4.log) lines"; done
wait $pid; rc=$?
echo "rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4.log) $(grep -o '"setup_s": [0-9.]*' $O/r4.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r4.log)"
