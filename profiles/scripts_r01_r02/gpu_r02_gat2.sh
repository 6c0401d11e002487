set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_gat2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cgnn_kernels_gpu.py -x -v -k "multi_device" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/products_fused_reordered.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 --reorder none > $O/products_fused_noreorder.log 2>&1 || exit 1
echo done
