set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_rbf
mkdir -p $O
V5=$PWD/variants/rbf5/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest tests/test_cgnn_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels_pow.log 2>&1 || exit 1
for rep in 1 2; do
for v in pow rbf5; do
  if [ $v = rbf5 ]; then export CGNN_HIP_LIB=$V5; else unset CGNN_HIP_LIB; fi
  timeout -k 10 120 python tools/bench_cgnn_batch.py --d 22 --edges 30 --R 256 --train 200 --test 100 >> $O/graph_$v.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 200 --test 100 >> $O/pair_$v.log 2>&1 || exit 1
done
done
unset CGNN_HIP_LIB
timeout -k 10 200 python examples/bench_cgnn_pairwise.py --data tests/data/Example_pairwise_pairs.csv > $O/pairwise_example_pow.log 2>&1 || exit 1
echo done
