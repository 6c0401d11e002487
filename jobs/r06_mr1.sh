#!/bin/bash
# Round 6: kernel sequence of one multi-rank GCN epoch (1/8-size graph, 1-rank nccl group,
# every exchange branch on) -- where the fills and copies come from
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mr1
mkdir -p $O
timeout -k 10 300 python -u tools/multirank_host.py > $O/host_gpu.log 2>&1 || { echo host probe failed; tail $O/host_gpu.log; exit 1; }
grep '^{' $O/host_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/multirank_host.py --forms collectives --epochs 10 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_kernels.py $O/prof/run_kernel_trace.csv 8 > $O/epoch_kernels.txt 2>&1 || true
cat $O/epoch_kernels.txt
echo done
