set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_long
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cgnn_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_long_n.py --N 100000 --d 2 --train 20 --test 10 > $O/long_pair_100k.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_long_n.py --N 100000 --d 10 --train 20 --test 10 > $O/long_dag10_100k.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_long_n.py --N 20000 --d 2 --train 50 --test 20 > $O/long_pair_20k.log 2>&1 || exit 1
echo done
