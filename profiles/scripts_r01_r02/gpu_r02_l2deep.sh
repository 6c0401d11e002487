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
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -n 20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 > $O/gat_papers_s0125.log 2>&1 || { echo "papers failed"; tail -n 20 $O/gat_papers_s0125.log; exit 1; }
tail -n 1 $O/gat_papers_s0125.log
echo l2deep-done
