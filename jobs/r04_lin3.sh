#!/bin/bash
# arxiv-shape dense kernels: kernel trace + PMC passes (write requests, instruction mix)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin3
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt.log 2>&1 || { echo "kt failed"; tail $O/kt.log; exit 1; }
grep '^{' $O/kt.log
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/pmc1 -o run -- python3 tools/bench_lin.py --shape arxiv --reps 2 > $O/pmc1.log 2>&1 || { echo "pmc1 failed"; tail $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 tools/bench_lin.py --shape arxiv --reps 2 > $O/pmc2.log 2>&1 || { echo "pmc2 failed"; tail $O/pmc2.log; exit 1; }
ls $O/pmc1 $O/pmc2
