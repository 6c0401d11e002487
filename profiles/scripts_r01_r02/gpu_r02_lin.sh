set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_lin
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_linear_gpu.py tests/test_gat_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 --steps 3 --warmup 1 > $O/sage.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/sprof -o run -- python -u tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py --top 30 /tmp/sprof/run_results.db > $O/sage_kernel_stats.csv
echo done
