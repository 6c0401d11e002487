#!/bin/bash
# Round 5: the fused layer-1 aggregation + dense forward (gnn_aggfwd.hip): bitwise tests
# against the two-kernel path, the benched composition, bench.py both ways, and a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_agg1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "agg_fwd or fused_aggregation or benched_config or fused_backward" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_fused.log 2>&1 || { echo bench failed; tail $O/bench_fused.log; exit 1; }
tail -n 1 $O/bench_fused.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-fuse-agg > $O/bench_two.log 2>&1 || { echo bench2 failed; tail $O/bench_two.log; exit 1; }
tail -n 1 $O/bench_two.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
echo done
