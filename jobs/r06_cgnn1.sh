#!/bin/bash
# Round 6: CGNN -- vectorized Adam, symmetric wide-MMD evaluation (in-tree) vs round 5
# (abv/cgnn_old): tests, batch step A/B at the orientation shape, full orientation run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_cgnn1
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/cgnn_old/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 600 python -u -m pytest tests/test_cgnn_kernels_gpu.py tests/test_cgnn_wide_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_new_$r.log 2>&1 || { echo batch failed; tail $O/batch_new_$r.log; exit 1; }
echo "new $r: $(tail -n 1 $O/batch_new_$r.log | cut -c1-300)"
CGNN_HIP_LIB=$OLD timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_old_$r.log 2>&1 || { echo batch failed; tail $O/batch_old_$r.log; exit 1; }
echo "old $r: $(tail -n 1 $O/batch_old_$r.log | cut -c1-300)"
done
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -q --timeout 200 --timeout-method thread -k "gcn or fused or ell" > $O/pytest_gcn.log 2>&1 \
    || { echo "gcn tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gcn.log | head -20; tail -n 30 $O/pytest_gcn.log; exit 1; }
tail -n 1 $O/pytest_gcn.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_$r.log 2>&1 || { echo bench failed; tail $O/bench_$r.log; exit 1; }
echo "bench $r: $(grep '^{' $O/bench_$r.log | cut -c80-160)"
done
timeout -k 10 500 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 1 $O/orient.log | cut -c1-400
echo done
