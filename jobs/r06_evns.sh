#!/bin/bash
# Round 6: evaluation steps skip storing the forward's noise draws (in-tree) vs HEAD; GraphSAGE sampler-only throughput
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_evns
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/head/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for v in new old; do
L=""; [ $v = old ] && L=$OLD
CGNN_HIP_LIB=$L timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_${v}_$r.log 2>&1 || { echo batch failed; tail $O/batch_${v}_$r.log; exit 1; }
echo "$v $r: $(tail -n 1 $O/batch_${v}_$r.log | cut -c100-260)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 50 --test 50 --eager > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06_evns/prof/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    if 'mmd' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
timeout -k 10 300 python -u tools/sage_sampler_only.py > $O/sampler_only.log 2>&1 || { echo sampler failed; tail $O/sampler_only.log; exit 1; }
grep "^{" $O/sampler_only.log
echo done
