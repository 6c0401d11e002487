#!/bin/bash
# Round 5: CGNN device-batch timing at the widths the round opened up (Fourier MMD > 256,
# exact MMD > 1024), and the d = 200 reference point
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_cgnn_time
mkdir -p $O
for spec in "200 400 --fast" "300 600 --fast" "512 1000 --fast" "1000 2000 --fast" "200 400" "1500 3000" "2048 4000"; do
  set -- $spec
  timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d $1 --edges $2 --R 32 --n 500 --train 20 --test 10 $3 >> $O/time.jsonl 2> $O/err_$1.log || { echo "d=$1 failed"; tail $O/err_$1.log; exit 1; }
  tail -n 1 $O/time.jsonl
done
echo done
