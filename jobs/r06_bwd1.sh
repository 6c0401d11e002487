#!/bin/bash
# Round 6: fused backward with 16x16x32 contractions (permlane16_swap A operands) vs the
# round-5 kernel (abv/dense_old): numerics tests, isolated kernel A/B, headline A/B, trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_bwd1
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/dense_old/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "ell or gcn or fused" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 200 python -u tools/ab_dense.py --iters 30 > $O/ab_new_$r.log 2>&1 || { echo ab new failed; tail $O/ab_new_$r.log; exit 1; }
CGNN_HIP_LIB=$OLD timeout -k 10 200 python -u tools/ab_dense.py --iters 30 > $O/ab_old_$r.log 2>&1 || { echo ab old failed; tail $O/ab_old_$r.log; exit 1; }
echo "new: $(grep '^{' $O/ab_new_$r.log)"; echo "old: $(grep '^{' $O/ab_old_$r.log)"
done
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_new_$r.log 2>&1 || { echo bench failed; tail $O/bench_new_$r.log; exit 1; }
CGNN_HIP_LIB=$OLD timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_old_$r.log 2>&1 || { echo bench failed; tail $O/bench_old_$r.log; exit 1; }
echo "new $r: $(grep '^{' $O/bench_new_$r.log | cut -c80-170)"; echo "old $r: $(grep '^{' $O/bench_old_$r.log | cut -c80-170)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
echo done
