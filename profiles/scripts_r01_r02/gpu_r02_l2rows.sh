#!/bin/bash
# Train-row-only layer-2 aggregation: GNN GPU tests, the headline bench with and
# without it (CGNN_L2_ALL_ROWS=1), its kernel-time profile, and a 2-rank full-scale
# one-GPU rehearsal (loss vs the one-rank run).  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/l2rows
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py tests/test_bench_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -n 20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
CGNN_L2_ALL_ROWS=1 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_allrows.log 2>&1 || { echo "bench allrows failed"; exit 1; }
tail -n 1 $O/bench_allrows.log
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/r1.log 2>&1 || { echo "r1 failed"; exit 1; }
timeout -k 10 420 python -u bench.py --gpus 2 --shared-gpu --steps 5 --warmup 2 > $O/r2.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "r2 running"; done
wait $pid; rc=$?
echo "r1 $(grep -o '"train_loss": [0-9.]*' $O/r1.log) r2 rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r2.log)"
[ $rc -eq 0 ] || exit 1
echo l2rows-done
timeout -k 10 420 python -u bench.py --gpus 4 --shared-gpu --steps 5 --warmup 2 > $O/r4.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "r4 running"; done
wait $pid; rc=$?
echo "r4 rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4.log)"
[ $rc -eq 0 ] || exit 1
echo r4-done
