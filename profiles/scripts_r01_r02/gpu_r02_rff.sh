set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_rff
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cgnn_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for v in mfma valu; do
  if [ $v = valu ]; then export CGNN_RFF_VALU=1; else unset CGNN_RFF_VALU; fi
  timeout -k 10 120 python tools/bench_cgnn_batch.py --d 22 --edges 30 --R 256 --train 200 --test 100 --fast >> $O/graph_fast_$v.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 200 --test 100 --fast >> $O/pair_fast_$v.log 2>&1 || exit 1
done
unset CGNN_RFF_VALU
CGNN_RFF_MFMA_MIN_D=1 timeout -k 10 120 python tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 200 --test 100 --fast >> $O/pair_fast_mfma_d2.log 2>&1 || exit 1
timeout -k 10 200 python examples/bench_cgnn_pairwise.py --data tests/data/Example_pairwise_pairs.csv --fast > $O/pairwise_example_fast.log 2>&1 || exit 1
timeout -k 10 200 python examples/bench_cgnn_pairwise.py --data tests/data/Example_pairwise_pairs.csv > $O/pairwise_example_exact.log 2>&1 || exit 1
cd examples
timeout -k 10 300 python run_CGNN_graph.py --out-dir ../$O --fast-mmd > ../$O/graph_example_fast.log 2>&1 || exit 1
timeout -k 10 300 python run_CGNN_graph.py --out-dir ../$O > ../$O/graph_example_exact.log 2>&1 || exit 1
echo done
