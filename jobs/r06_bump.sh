#!/bin/bash
# Round 6: GraphSAGE step counter advanced by the bias-gradient reduction (no add launch) vs the separate add
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_bump
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_sampler_gpu.py tests/test_gnn_linear_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2 3; do
for v in 1 0; do
CGNN_SAGE_BUMP=$v timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_${v}_$r.log 2>&1 || { echo sage failed; tail $O/sage_${v}_$r.log; exit 1; }
echo "bump $v run $r: $(grep -o '"value": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_${v}_$r.log) $(grep -o '"train_loss": [0-9.]*' $O/sage_${v}_$r.log)"
done
done
echo done
