#!/bin/bash
# Round 6: layer-1 features as a split table (192-B main rows + 16-B tail rows) vs 256-B rows
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_split
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "split or benched_config or spmm_matches or ell" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_spmm_width.py > $O/width.log 2>&1 || { echo width failed; tail $O/width.log; exit 1; }
cat $O/width.log
for r in 1 2; do
for t in split dense; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --x-table $t > $O/bench_${t}_$r.log 2>&1 || { echo bench failed; tail $O/bench_${t}_$r.log; exit 1; }
echo "$t $r: $(grep -o '"value": [0-9.]*' $O/bench_${t}_$r.log) $(grep -o '"val_acc": [0-9.]*' $O/bench_${t}_$r.log)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
echo done
