#!/bin/bash
# Round 5: fused aggregation variants (U = 16 / 8 rows in flight per lane; gather only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_agg2
mkdir -p $O
timeout -k 10 200 python -u tools/ab_agg.py > $O/ab_default.log 2>&1 || { echo ab failed; tail $O/ab_default.log; exit 1; }
tail -n 1 $O/ab_default.log
for v in v_gonly v_u8 v_u8g v_lw8 v_lw8g; do
  CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so timeout -k 10 200 python -u tools/ab_agg.py --only-agg > $O/ab_$v.log 2>&1 || { echo ab $v failed; tail $O/ab_$v.log; exit 1; }
  tail -n 1 $O/ab_$v.log
done
timeout -k 10 200 python -u tools/ab_agg.py > $O/ab_default2.log 2>&1 || { echo ab failed; tail $O/ab_default2.log; exit 1; }
tail -n 1 $O/ab_default2.log
