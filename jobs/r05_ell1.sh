#!/bin/bash
# Round 5: the backward's train-column aggregation (spmm_ell): 1 / 2 rows per sub-group, persistent pipelined
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ell1
mkdir -p $O
for r in 1 2; do
for v in default e_rp2 e_pipe6 e_pipe14; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so; fi
  timeout -k 10 200 python -u tools/ab_agg.py --only-ell > $O/ab_${v}_$r.log 2>&1 || { echo ab $v failed; tail $O/ab_${v}_$r.log; exit 1; }
  tail -n 1 $O/ab_${v}_$r.log
done
done
unset CGNN_HIP_LIB
echo done
