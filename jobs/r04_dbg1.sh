#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dbg1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gnn_gpu.py > $O/tests.log 2>&1
grep -E "FAILED|passed|failed" $O/tests.log | tail -n 20
exit 0
