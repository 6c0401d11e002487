#!/bin/bash
# Round 5: layer-1 spmm with 16 rows in flight per lane / DPP id broadcast
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_spmm1
mkdir -p $O
for r in 1 2; do
for v in default s_u16 s_dpp; do
  if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so; fi
  timeout -k 10 200 python -u tools/ab_agg.py --only-spmm > $O/ab_${v}_$r.log 2>&1 || { echo ab $v failed; tail $O/ab_${v}_$r.log; exit 1; }
  tail -n 1 $O/ab_${v}_$r.log
done
done
unset CGNN_HIP_LIB
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM --kernel-include-regex "spmm_kernel" --output-format csv -d $O/pmc -o run -- python3 tools/ab_agg.py --iters 2 --only-spmm > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }

timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_wide.log 2>&1 \
    || { echo "wide tests failed"; grep -E "FAILED|Error|assert" $O/pytest_wide.log | head -20; tail -n 30 $O/pytest_wide.log; exit 1; }
tail -n 1 $O/pytest_wide.log
echo done
