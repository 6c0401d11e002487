#!/bin/bash
# Wide CGNN after the level-scheduled kernels: tests, d = 200 batch benches, kernel
# profile, and CGNN().orient_directed_graph on RandomGraphGenerator(200) data at the
# reference settings (time-boxed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_wide2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_cgnn_wide_gpu.py tests/test_cgnn_kernels_gpu.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for cfg in "20 256" "100 256" "100 32" "20 32"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R $2 --n 500 --h $1 --train 50 --test 20 > $O/d200_h$1_r$2.log 2>&1 || { echo "bench h$1 r$2 failed"; tail $O/d200_h$1_r$2.log; exit 1; }
  tail -n 1 $O/d200_h$1_r$2.log
done
for h in 20 100; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$h -o run -- python3 -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 256 --n 500 --h $h --train 20 --test 10 --eager > $O/prof$h.log 2>&1 || { echo prof failed; tail $O/prof$h.log; exit 1; }
python3 - $h <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/r04_wide2/prof%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True)
for r in list(csv.DictReader(open(f[0])))[:7]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
done
find $O -name "*_trace.csv" -delete
timeout -k 10 420 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail -20 $O/orient.log; exit 1; }
tail -n 1 $O/orient.log
echo done
