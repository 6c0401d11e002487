#!/bin/bash
# Fresh-box validation after the container rebuild: GPU tests, smoke(), the headline
# bench, and a full-scale 4-rank one-GPU rehearsal with the default (overlapped)
# backward schedule.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 3 $O/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -n 20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 \
    || { echo "bench failed"; tail -n 20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -k 10 420 python -u bench.py --gpus 4 --shared-gpu --steps 5 --warmup 2 > $O/r4.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "r4 running $(wc -l < $O/r4.log) lines"; done
wait $pid; rc=$?
echo "r4 rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r4.log)"
[ $rc -eq 0 ] || exit 1
echo final4-done
