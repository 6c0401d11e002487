set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_gcn3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py tests/test_gnn_linear_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/bench_fused.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_gnn_configs.py --config arxiv-gcn3 --unfused > $O/bench_unfused.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_gnn_configs.py --config arxiv-gcn3 --reorder none > $O/bench_fused_noreorder.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config arxiv-gcn3 --no-capture --steps 50 > $O/trace.log 2>&1 || exit 1
echo done
