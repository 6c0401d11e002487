set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_examples
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_examples_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u examples/run_GNN_pairwise_inference.py --out-dir $O > $O/pairwise.log 2>&1 || exit 1
timeout -k 10 300 python -u examples/run_CGNN_graph.py --out-dir $O > $O/graph.log 2>&1 || exit 1
timeout -k 10 300 python -u examples/run_CGNN_graph_hidden_variables.py --out-dir $O > $O/conf.log 2>&1 || exit 1
echo done
