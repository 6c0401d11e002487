#!/bin/bash
# Round 3: new GAT kernels (no-gather row half, batched gathers, fused activation,
# bf16 dy in place) and the wide-CGNN path: GPU tests, products epoch, kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_gatv2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -k "gat or fused or gcn_benched" -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gat.log 2>&1 || { echo "pytest gat failed"; tail -n 40 $O/pytest_gat.log; exit 1; }
tail -n 2 $O/pytest_gat.log
timeout -k 10 300 python3 -u tools/bench_gat.py --steps 10 --warmup 2 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_gat.py --steps 5 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 tools/pmc_summary.py --trace $O/trace --top 14 > $O/summary.md 2>&1
cat $O/summary.md
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_cgnn.log 2>&1 || { echo "pytest cgnn failed"; tail -n 40 $O/pytest_cgnn.log; exit 1; }
tail -n 2 $O/pytest_cgnn.log
echo done
