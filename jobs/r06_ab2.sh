#!/bin/bash
# Round 6: AX row pitch 104 vs 128 on the dense kernels; eval-MMD kernel time new vs old
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ab2
mkdir -p $O
OLD=$GRAFT_REPO_ROOT/abv/cgnn_old/_hip.cpython-310-x86_64-linux-gnu.so
for r in 1 2; do
for l in 104 128; do
timeout -k 10 200 python -u tools/ab_dense.py --iters 30 --ldx $l > $O/ab_ldx${l}_$r.log 2>&1 || { echo ab failed; tail $O/ab_ldx${l}_$r.log; exit 1; }
echo "ldx $l: $(grep '^{' $O/ab_ldx${l}_$r.log | cut -c1-120)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pnew -o run -- python3 tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 20 --test 20 --eager > $O/pnew.log 2>&1 || { echo prof failed; tail $O/pnew.log; exit 1; }
CGNN_HIP_LIB=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pold -o run -- python3 tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 20 --test 20 --eager > $O/pold.log 2>&1 || { echo prof failed; tail $O/pold.log; exit 1; }
for v in pnew pold; do echo $v; head -8 $O/$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150; done
find $O -name "*kernel_trace.csv" -delete
echo done
