#!/bin/bash
# Round 5: what bounds the transposed aggregation (short rows): timings + PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_short2
mkdir -p $O
timeout -k 10 300 python -u tools/ab_short.py > $O/ab.log 2>&1 || { echo ab failed; tail $O/ab.log; exit 1; }
tail -n 2 $O/ab.log
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/$O/p1 -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_short.py > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 || { echo p1 failed; tail $GRAFT_REPO_ROOT/$O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/p2 -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_short.py > $GRAFT_REPO_ROOT/$O/p2.log 2>&1 || { echo p2 failed; tail $GRAFT_REPO_ROOT/$O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $GRAFT_REPO_ROOT/$O/p3 -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_short.py > $GRAFT_REPO_ROOT/$O/p3.log 2>&1 || { echo p3 failed; tail $GRAFT_REPO_ROOT/$O/p3.log; exit 1; }
echo done
