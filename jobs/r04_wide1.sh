#!/bin/bash
# Round 4: (1) re-pin the example gates (confounders at 32 runs) + compat_scores record;
# (2) wide CGNN (d = 200, the random-graph generator's default) kernel profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_wide1
mkdir -p $O
timeout -k 10 400 python -u tools/pin_examples.py $O/expected_examples.json > $O/pin.log 2>&1 || { echo pin failed; tail -20 $O/pin.log; exit 1; }
tail -n 1 $O/pin.log
timeout -k 10 400 python -u tools/pin_examples.py --compat $O/compat_examples.json > $O/pin_compat.log 2>&1 || { echo compat failed; tail -20 $O/pin_compat.log; exit 1; }
tail -n 1 $O/pin_compat.log
for cfg in "20 256" "20 32" "100 32"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R $2 --n 500 --h $1 --train 50 --test 20 > $O/d200_h$1_r$2.log 2>&1 || { echo "bench h$1 r$2 failed"; tail $O/d200_h$1_r$2.log; exit 1; }
  tail -n 1 $O/d200_h$1_r$2.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 256 --n 500 --h 20 --train 20 --test 10 --eager > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04_wide1/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:12]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
find $O -name "*_trace.csv" -delete
echo done
