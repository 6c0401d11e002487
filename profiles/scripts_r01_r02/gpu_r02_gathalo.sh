#!/bin/bash
# Training halo of the sharded fused GAT: GPU tests (sharded over ranks on one GPU)
# and the papers100M full-size rank-0-of-8 dry run.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gathalo
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gat_fused_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gat.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest_gat.log; exit 1; }
tail -n 2 $O/pytest_gat.log
timeout -k 10 600 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 1.0 --steps 3 --warmup 1 --emulate-world 8 > $O/gat_emulate_r0of8_full.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; kill -0 $pid 2>/dev/null && echo "emulate running"; done
wait $pid; rc=$?
tail -n 1 $O/gat_emulate_r0of8_full.log
[ $rc -eq 0 ] || exit 1
echo gathalo-done
