#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/slab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench$r.log 2>&1 || exit 1
  echo "bench $(grep -o '"value": [0-9.]*' $O/bench$r.log) $(grep -o '"train_loss": [0-9.]*' $O/bench$r.log)"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "rocprof failed"; exit 1; }
bash profiles/scripts_r01_r02/gpu_rehearse.sh
