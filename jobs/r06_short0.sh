#!/bin/bash
# Round 6: GraphSAGE forward aggregations on the short-row kernel (4 rows per sub-group) vs the one-row kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_short0
mkdir -p $O
for r in 1 2; do
for v in none 0 01; do
E="CGNN_SAGE_SHORTX=0"; [ $v = 0 ] && E="CGNN_SAGE_SHORT0=1"; [ $v = 01 ] && E="CGNN_SAGE_SHORT0=1 CGNN_SAGE_SHORT1=1"
env $E timeout -k 10 300 python -u tools/sage_train_only.py --steps 192 > $O/to_${v}_$r.log 2>&1 || { echo failed; tail $O/to_${v}_$r.log; exit 1; }
echo "$v $r: $(grep -o '"train_only_us_per_step": [0-9.]*' $O/to_${v}_$r.log)"
done
done
CGNN_SAGE_SHORT0=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/sage_train_only.py --steps 32 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
grep -i "spmm" $O/prof/run_kernel_stats.csv | cut -c1-160
echo done
