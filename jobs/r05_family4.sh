#!/bin/bash
# Round 5: per-sample vs level-scheduled generator after the staged-backward changes
# (d = 12 .. 28, 30 edges per 22 variables scaled, R = 256, N = 500, H = 20)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_family4
mkdir -p $O
for d in ${DS:-12 16 22 28}; do
  e=$(( d * 30 / 22 ))
  for g in auto staged; do
    timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d $d --edges $e --generator $g > $O/d${d}_$g.log 2>&1 || { echo d$d $g failed; tail $O/d${d}_$g.log; exit 1; }
    echo $d $g $(grep '^{' $O/d${d}_$g.log | cut -c1-260)
  done
done
echo done
