#!/bin/bash
# Round 6: software-pipelined fused backward (in-tree: tile i+1's epilogue beside tile i's
# contractions, weights in LDS) vs the 16x16 kernel without the pipeline (abv/dense_v1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_bwd3
mkdir -p $O
V1=$GRAFT_REPO_ROOT/abv/dense_v1/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "ell or gcn or fused" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for v in new v1; do
L=""; [ $v = v1 ] && L=$V1
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
echo done
