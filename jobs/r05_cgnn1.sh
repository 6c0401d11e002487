#!/bin/bash
# Round 5: wide Fourier MMD, exact MMD beyond 1024, multi-device / shared-GPU scorer tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_cgnn1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cgnn_kernels_gpu.py tests/test_cgnn_wide_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
grep -E "PASSED|FAILED" $O/pytest.log | grep -E "wide_form|fast_mmd|beyond_1024|multi_device|sharing|independent" 
echo done
