#!/bin/bash
# Round 3 GAT baseline: products epoch time, kernel trace, and two PMC passes on the
# attention-aggregation kernels.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_gat
mkdir -p $O
B="python3 tools/bench_gat.py --steps 5 --warmup 1"
timeout -k 10 300 python3 -u tools/bench_gat.py --steps 10 --warmup 2 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_ANY FETCH_SIZE --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || { echo pmca failed; tail $O/pmca.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || { echo pmcb failed; tail $O/pmcb.log; exit 1; }
python3 tools/pmc_summary.py --trace $O/trace --pmc $O/pmc_a $O/pmc_b --top 16 > $O/summary.md 2>&1
cat $O/summary.md
echo done
