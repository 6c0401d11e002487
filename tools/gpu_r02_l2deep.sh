#!/bin/bash
# Train-row last layer in the L-layer GCN: GPU tests, arxiv 3-layer epoch with /
# without it.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/l2deep
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py tests/test_checks_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo "arxiv failed"; tail -n 20 $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log
CGNN_L2_ALL_ROWS=1 timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_allrows.log 2>&1 || { echo "arxiv allrows failed"; exit 1; }
tail -n 1 $O/arxiv_allrows.log
echo l2deep-done
