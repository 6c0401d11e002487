#!/bin/bash
# Layer 1 at the train-neighbour rows in training: GNN GPU tests, the headline with /
# without it, a 4-rank one-GPU rehearsal.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/l1nbrs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py tests/test_bench_gpu.py tests/test_checks_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in "nbrs:1" "all:0"; do
  name=${v%%:*}; val=${v#*:}
  CGNN_L1_TRAIN_NBRS=$val timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_$name.log 2>&1 || { echo "bench $name failed"; tail -n 20 $O/bench_$name.log; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$name.log) $(grep -o '"train_loss": [0-9.]*' $O/bench_$name.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_$name.log)"
done
timeout -k 10 420 python -u bench.py --gpus 4 --shared-gpu --steps 5 --warmup 2 > $O/r4.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "r4 running"; done
wait $pid; rc=$?
echo "r4 rc=$rc $(grep -o '"train_loss": [0-9.]*' $O/r4.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/r1.log 2>&1 || exit 1
echo "r1 $(grep -o '"train_loss": [0-9.]*' $O/r1.log)"
echo l1nbrs-done
