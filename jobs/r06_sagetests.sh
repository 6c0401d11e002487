#!/bin/bash
# Round 6: GraphSAGE / sampler GPU tests on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sagetests
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_sampler_gpu.py tests/test_checks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
echo done
