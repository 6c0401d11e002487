#!/bin/bash
# A/B: one-GPU GCN epoch with the layer-1 aggregation of the next epoch on a side stream
# (default) vs in line (CGNN_AX_PIPELINE=0); plus the exactness test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -k "pipeline or spmm_win" -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  CGNN_AX_PIPELINE=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_pipe$v.log 2>&1 || exit 1
  echo "pipe=$v $(grep -o '"value": [0-9.]*' $O/bench_pipe$v.log) $(grep -o '"train_loss": [0-9.]*' $O/bench_pipe$v.log)"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
