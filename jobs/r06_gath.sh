#!/bin/bash
# Round 6: fused backward with the train-column aggregate gathered in-kernel (no ELL launch, no dY2 round trip)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_gath
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "gather_bitwise or fused_backward or benched_config or ell" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for v in gather ell; do
A=""; [ $v = ell ] && A="--no-bwd-gather"
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 $A > $O/bench_${v}_$r.log 2>&1 || { echo bench failed; tail $O/bench_${v}_$r.log; exit 1; }
echo "bench $v $r: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_${v}_$r.log)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_kernels.py $O/prof/run_kernel_trace.csv > $O/epoch_kernels.txt 2>&1 || true
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt $O/epoch_kernels.txt | head -40
echo done
