#!/bin/bash
# Round 6: staggered fused backward (in-tree) vs 16x16 without stagger (abv/dense_v1) vs
# round 5 (abv/dense_old); XCD-local ELL aggregation; trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_bwd2
mkdir -p $O
V1=$GRAFT_REPO_ROOT/abv/dense_v1/_hip.cpython-310-x86_64-linux-gnu.so
OLD=$GRAFT_REPO_ROOT/abv/dense_old/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "ell or gcn or fused" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for v in new v1 old; do
L=""; [ $v = v1 ] && L=$V1; [ $v = old ] && L=$OLD
CGNN_HIP_LIB=$L timeout -k 10 200 python -u tools/ab_dense.py --iters 30 > $O/ab_${v}_$r.log 2>&1 || { echo ab $v failed; tail $O/ab_${v}_$r.log; exit 1; }
echo "$v: $(grep '^{' $O/ab_${v}_$r.log | cut -c1-140)"
done
done
for r in 1 2; do
for v in new v1; do
L=""; [ $v = v1 ] && L=$V1
CGNN_HIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_${v}_$r.log 2>&1 || { echo bench failed; tail $O/bench_${v}_$r.log; exit 1; }
echo "$v $r: $(grep '^{' $O/bench_${v}_$r.log | cut -c80-150)"
done
done
CGNN_ELL_FORM=0 timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_ell0.log 2>&1 || { echo bench failed; tail $O/bench_ell0.log; exit 1; }
echo "new ell0: $(grep '^{' $O/bench_ell0.log | cut -c80-150)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
echo done
