#!/bin/bash
# Round 5: the whole GPU test suite after the SAGE / short-row SpMM / GAT remap / Fourier
# threshold changes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_gpu_suite1
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -20
tail -n 2 $O/pytest.log
exit $rc
