#!/bin/bash
# Round 6: pipelined SpMM for sampled blocks of fanout <= 8 (SAGE input layer) -- tests, training-only step, SAGE bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_fan
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_sampler_gpu.py -x -v --timeout 300 --timeout-method thread -k "fan or sage or sampler or spmm" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/sage_train_only.py --steps 192 > $O/to_$r.log 2>&1 || { echo failed; tail $O/to_$r.log; exit 1; }
echo "train-only $r: $(grep -o '"train_only_us_per_step": [0-9.]*' $O/to_$r.log)"
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
echo "sage $r: $(grep -o '"value": [0-9.]*' $O/sage_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/sage_train_only.py --steps 32 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
grep -i "spmm" $O/prof/run_kernel_stats.csv | cut -c1-150
echo done
