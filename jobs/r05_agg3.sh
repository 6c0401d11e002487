#!/bin/bash
# Round 5: is the persistent gather's loss its row window?  gather-only with 4/8/16/32 rows
# per dequeue, and L2 hit counters of spmm vs the fused kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_agg3
mkdir -p $O
for v in v_gonly v_gt16g v_gt8g v_gt4g; do
  CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so timeout -k 10 200 python -u tools/ab_agg.py --only-agg > $O/ab_$v.log 2>&1 || { echo ab $v failed; tail $O/ab_$v.log; exit 1; }
  tail -n 1 $O/ab_$v.log
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex "spmm_kernel|gcn_agg" --output-format csv -d $O/pmc -o run -- python3 tools/ab_agg.py --iters 2 > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
CGNN_HIP_LIB=$PWD/abtmp/_hip_v_gt8g.so timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex "gcn_agg" --output-format csv -d $O/pmc8 -o run -- python3 tools/ab_agg.py --iters 2 --only-agg > $O/pmc8.log 2>&1 || { echo pmc8 failed; tail $O/pmc8.log; exit 1; }
echo done
