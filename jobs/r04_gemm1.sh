#!/bin/bash
# lin_gemm: staging registers as named scalars (no scratch), loads pinned ahead of the MFMAs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_gemm1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_linear_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_kt -o run -- python3 tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_kt.log 2>&1 || { echo "reddit kt failed"; tail $O/reddit_kt.log; exit 1; }
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit.log 2>&1 || { echo "reddit failed"; tail $O/reddit.log; exit 1; }
tail -n 1 $O/reddit.log | cut -c1-200
find $O -name "*_trace.csv" -delete
