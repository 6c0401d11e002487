set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_gatfused
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -x -v -k gat --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/products_fused.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 --unfused > $O/products_unfused.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_products -o run -- python -u tools/bench_gat.py --steps 5 --warmup 1 > $O/prof_products.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 > $O/gat_world1_s0125.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 --unfused > $O/gat_world1_s0125_unfused.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 1.0 --steps 3 --warmup 1 --emulate-world 8 > $O/gat_emulate_r0of8_full.log 2>&1 || exit 1
echo done
