#!/bin/bash
# Round 6: CGNN -- 16-B column-tile staging in the wide MMD + vectorized Adam (in-tree) vs
# round 5 (abv/cgnn_old): tests, batch A/B, kernel profile, orientation run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_cgnn2
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/cgnn_old/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 600 python -u -m pytest tests/test_cgnn_kernels_gpu.py tests/test_cgnn_wide_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_new_$r.log 2>&1 || { echo batch failed; tail $O/batch_new_$r.log; exit 1; }
echo "new $r: $(tail -n 1 $O/batch_new_$r.log | cut -c100-260)"
CGNN_HIP_LIB=$OLD timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_old_$r.log 2>&1 || { echo batch failed; tail $O/batch_old_$r.log; exit 1; }
echo "old $r: $(tail -n 1 $O/batch_old_$r.log | cut -c100-260)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pnew -o run -- python3 tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 20 --test 20 --eager > $O/pnew.log 2>&1 || { echo prof failed; tail $O/pnew.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/pnew/run_kernel_stats.csv')):
    print('%-60s %6s %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" | head -8
find $O -name "*kernel_trace.csv" -delete
timeout -k 10 500 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 1 $O/orient.log | cut -c1-400
echo done
