#!/bin/bash
# Round 5: CGNN GPU tests after the generator family threshold moved to 24 variables
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_family_tests
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py tests/test_examples_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
   || { echo tests failed; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -n 20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
echo done
