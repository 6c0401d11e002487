#!/bin/bash
# Round 5: matrix-core vs vector MMD at small widths (the example scripts' d = 19 / 22)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_mmdchoice
mkdir -p $O
for spec in "8 10 0" "12 16 0" "19 40 3" "22 30 0" "30 45 0"; do
  set -- $spec
  for k in mfma valu; do
    CGNN_MMD_KERNEL=$k timeout -k 10 200 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --conf $3 --R 256 --n 500 --h 20 --train 100 --test 50 > $O/tmp.log 2> $O/err.log || { echo "d=$1 $k failed"; tail $O/err.log; exit 1; }
    echo "{\"mmd\": \"$k\", \"res\": $(tail -n 1 $O/tmp.log)}" >> $O/mmd.jsonl
    tail -n 1 $O/mmd.jsonl | cut -c1-300
  done
done
echo done
