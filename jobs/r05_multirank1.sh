#!/bin/bash
# Round 5: host:GPU ratio of a 1/8-size multi-rank GCN epoch on a
# 1-rank nccl group, and a 2-rank --shared-gpu papers-gat2 rehearsal at scale 0.1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_multirank1
mkdir -p $O
timeout -k 10 400 python -u tools/multirank_host.py > $O/host_gpu.log 2>&1 || { echo host probe failed; tail $O/host_gpu.log; exit 1; }
grep '^{' $O/host_gpu.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
   tools/bench_gnn_configs.py --config papers-gat2 --scale 0.1 --shared-gpu --steps 3 --warmup 1 > $O/papers_rehearsal.log 2>&1 \
   || { echo rehearsal failed; tail -n 30 $O/papers_rehearsal.log; exit 1; }
grep '^{' $O/papers_rehearsal.log | cut -c1-600
echo done
