#!/bin/bash
# Round 6: GNN Adam increments its own step counter (no add launch); SAGE loss sums (no division launch)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_adamfold
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_sampler_gpu.py tests/test_gat_fused_gpu.py tests/test_gnn_linear_gpu.py tests/test_checks_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2 3; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
echo "sage $r: $(grep -o '"value": [0-9.]*' $O/sage_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_$r.log) $(grep -o '"train_loss": [0-9.]*' $O/sage_$r.log)"
done
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_$r.log 2>&1 || { echo bench failed; tail $O/bench_$r.log; exit 1; }
echo "bench $r: $(grep -o '"value": [0-9.]*' $O/bench_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_$r.log)"
done
echo done
