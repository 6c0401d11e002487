#!/bin/bash
# Round 6: static s_setprio for waves 4-7 in the fused GCN backward and the wide MMD
# (in-tree) vs HEAD (abv/head)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_prio
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/head/_hip.cpython-310-x86_64-linux-gnu.so
for r in 1 2; do
for v in new old; do
L=""; [ $v = old ] && L=$OLD
CGNN_HIP_LIB=$L timeout -k 10 200 python -u tools/ab_dense.py --iters 30 --ldx 104 > $O/ab_${v}_$r.log 2>&1 || { echo ab failed; tail $O/ab_${v}_$r.log; exit 1; }
echo "$v: $(grep '^{' $O/ab_${v}_$r.log | cut -c1-120)"
CGNN_HIP_LIB=$L timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 100 --test 100 > $O/batch_${v}_$r.log 2>&1 || { echo batch failed; tail $O/batch_${v}_$r.log; exit 1; }
echo "$v $r: $(tail -n 1 $O/batch_${v}_$r.log | cut -c100-220)"
done
done
echo done
