#!/bin/bash
# Round 6 closing check after the SAGE loss-sum and step-bump changes: whole GPU suite, smoke, headline bench, SAGE
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
echo "sage: $(grep -o '"value": [0-9.]*' $O/sage.log) $(grep -o '"val_acc": [0-9.]*' $O/sage.log)"
echo done
