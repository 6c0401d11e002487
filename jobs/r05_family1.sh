#!/bin/bash
# Round 5: per-sample vs level-scheduled generator kernels at small widths (the example
# scripts' d = 19 / 22 and up): where should the kernel family switch?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_family1
mkdir -p $O
for spec in "19 40 3" "22 30 0" "40 80 0" "64 128 0" "100 200 0"; do
  set -- $spec
  for gen in auto staged; do
    timeout -k 10 200 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --conf $3 --R 256 --n 500 --h 20 --train 100 --test 50 --generator $gen >> $O/family.jsonl 2> $O/err.log || { echo "d=$1 $gen failed"; tail $O/err.log; exit 1; }
    tail -n 1 $O/family.jsonl | cut -c1-260
  done
done
echo done
