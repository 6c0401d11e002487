#!/bin/bash
# Round 5: next epoch's layer-1 SpMM on a side stream beside the layer-2 / backward chain
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_pref1
mkdir -p $O
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "prefetched or benched_config or fused_aggregation" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$r.log 2>&1 || { echo bench failed; tail $O/bench_$r.log; exit 1; }
tail -n 1 $O/bench_$r.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
tail -n 20 $O/epoch_trace.txt
echo done
