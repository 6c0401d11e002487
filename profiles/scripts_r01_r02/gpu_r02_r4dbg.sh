#!/bin/bash
# 4-rank one-GPU rehearsal (gloo, blocking device collectives) with periodic stack
# dumps, then the bench GPU tests.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4dbg2
mkdir -p $O
CGNN_TRACEBACK_AFTER=60 timeout -k 10 360 python -u bench.py --gpus 4 --shared-gpu --steps 5 --warmup 2 > $O/r4.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "r4 running $(wc -l < $O/r4.log)"; done
wait $pid; rc=$?
echo "r4 rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r4.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_bench.log 2>&1 || { tail -n 20 $O/pytest_bench.log; exit 1; }
tail -n 2 $O/pytest_bench.log
echo r4dbg2-done
