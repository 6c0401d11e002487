#!/bin/bash
# Round 5: PMC of the staged CGNN backward after the register / MFMA change, and the
# reference-settings orientation run (time_orient) to see where it stands against 180 s
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_cgnnbwd3
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $GRAFT_REPO_ROOT/$O/p1 -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_staged.py --d 200 --edges 400 --R 256 --n 500 --h 20 --only bwd:4:2 --reps 3 > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 || { echo p1 failed; tail $GRAFT_REPO_ROOT/$O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/$O/p2 -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_staged.py --d 200 --edges 400 --R 256 --n 500 --h 20 --only bwd:4:2 --reps 3 > $GRAFT_REPO_ROOT/$O/p2.log 2>&1 || { echo p2 failed; tail $GRAFT_REPO_ROOT/$O/p2.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 1 $O/orient.log | cut -c1-500
echo done
