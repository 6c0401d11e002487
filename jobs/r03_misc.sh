#!/bin/bash
# Round 3: fused backward TB=2 vs TB=1 after the epilogue rewrite; the per-rank proxy of an
# 8-rank epoch (a 1/8-size graph on one GPU), eager vs hipGraph replay there and at full size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_misc
mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail $O/$name.log; exit 1; }; echo "$name $(tail -n 1 $O/$name.log | cut -c1-170)"; }
run tb1 env CGNN_FUSED_BWD_TB=1 python -u bench.py --steps 40 --warmup 5
run tb2 env CGNN_FUSED_BWD_TB=2 python -u bench.py --steps 40 --warmup 5
run full_capture python -u bench.py --steps 40 --warmup 5 --capture
run s0125 python -u bench.py --steps 100 --warmup 10 --scale 0.125
run s0125_capture python -u bench.py --steps 100 --warmup 10 --scale 0.125 --capture
run cgnn_d22 python -u tools/bench_cgnn_batch.py --d 22 --edges 30 --R 256 --train 200 --test 100
run cgnn_d100 python -u tools/bench_cgnn_batch.py --d 100 --edges 200 --R 64 --n 500 --h 25 --train 100 --test 50
run cgnn_d200 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 32 --n 500 --h 100 --train 50 --test 20
echo done
