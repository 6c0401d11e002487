#!/bin/bash
# Round 6: fused backward as two 4-wave blocks per CU (hidden halves, independent barriers; HS=2) vs one 8-wave block (HS=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_hs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "fused_backward or benched_config or gcn_steps" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for v in 2 1; do
CGNN_BWD_HS=$v timeout -k 10 200 python -u tools/ab_dense.py --iters 30 --ldx 104 > $O/ab_hs${v}_$r.log 2>&1 || { echo ab failed; tail $O/ab_hs${v}_$r.log; exit 1; }
echo "hs$v: $(grep '^{' $O/ab_hs${v}_$r.log | cut -c1-150)"
done
done
for r in 1 2; do
for v in 2 1; do
CGNN_BWD_HS=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_hs${v}_$r.log 2>&1 || { echo bench failed; tail $O/bench_hs${v}_$r.log; exit 1; }
echo "bench hs$v $r: $(grep -o '"value": [0-9.]*' $O/bench_hs${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_hs${v}_$r.log)"
done
done
echo done
