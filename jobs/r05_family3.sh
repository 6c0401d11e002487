#!/bin/bash
# Round 5: the per-sample / level-scheduled crossover between 22 and 40 variables
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_family3
mkdir -p $O
for spec in "24 48" "26 52" "28 56" "30 60" "32 64"; do
  set -- $spec
  for gen in auto staged; do
    timeout -k 10 200 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --R 256 --n 500 --h 20 --train 100 --test 50 --generator $gen >> $O/family.jsonl 2> $O/err.log || { echo "d=$1 $gen failed"; tail $O/err.log; exit 1; }
    tail -n 1 $O/family.jsonl | cut -c1-200
  done
done
echo done
