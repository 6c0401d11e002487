#!/bin/bash
# Round 6: GraphSAGE sampler with the collapsed launch chain (in-tree) vs round 5 (abv/sampler_old)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sage1
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/sampler_old/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_sampler_gpu.py tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread -k "sage or sampler" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_new_$r.log 2>&1 || { echo sage failed; tail $O/sage_new_$r.log; exit 1; }
echo "new $r: $(tail -n 1 $O/sage_new_$r.log | cut -c1-220)"
CGNN_HIP_LIB=$OLD timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_old_$r.log 2>&1 || { echo sage failed; tail $O/sage_old_$r.log; exit 1; }
echo "old $r: $(tail -n 1 $O/sage_old_$r.log | cut -c1-220)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
find $O/trace -name "*kernel_trace.csv" -delete
echo done
