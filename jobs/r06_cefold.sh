#!/bin/bash
# Round 6: the CE stats reduction writes gb2 directly (no copy launch) -- GNN GPU tests, headline bench x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_cefold
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_rccl_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_$r.log 2>&1 || { echo bench failed; tail $O/bench_$r.log; exit 1; }
echo "bench $r: $(grep -o '"value": [0-9.]*' $O/bench_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_$r.log) $(grep -o '"train_loss": [0-9.]*' $O/bench_$r.log)"
done
timeout -k 10 300 python -u tools/multirank_host.py > $O/host_gpu.log 2>&1 || { echo host probe failed; tail $O/host_gpu.log; exit 1; }
grep '^{' $O/host_gpu.log | cut -c1-200
echo done
