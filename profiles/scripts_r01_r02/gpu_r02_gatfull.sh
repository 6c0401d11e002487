set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_gatfull
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -x -v -k gat --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 1.0 --steps 3 --warmup 1 --emulate-world 8 > $O/gat_emulate_r0of8_full.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 > $O/gat_world1_s0125.log 2>&1 || exit 1
echo done
