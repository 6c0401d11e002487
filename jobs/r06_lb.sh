#!/bin/bash
# Round 6: sampler launch chain with single-pass look-back scans (4 launches per level, 7 transposed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_lb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sampler_gpu.py tests/test_gnn_gpu.py -x -v --timeout 300 --timeout-method thread -k "sampler or sage" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/sage_sampler_only.py > $O/sampler_only.log 2>&1 || { echo sampler failed; tail $O/sampler_only.log; exit 1; }
grep "^{" $O/sampler_only.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
echo "sage $r: $(grep -o '"value": [0-9.]*' $O/sage_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/sage_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/sage_trace.py $O/prof > $O/sage_trace.txt 2>&1 || true
head -8 $O/sage_trace.txt
find $O/prof -name "*kernel_trace.csv" -delete
grep -E "sb_|sample_neighbors" $O/prof/run_kernel_stats.csv | cut -c1-120
echo done
