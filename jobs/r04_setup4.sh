#!/bin/bash
# bench.py with 4 ranks sharing the one GPU (gloo collectives): the multi-rank setup cost
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_setup4
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.log; done) &
HB=$!
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 10 --warmup 3 --shared-gpu > $O/bench4.log 2>&1
rc=$?
kill $HB
grep -v amdgpu.ids $O/bench4.log | tail -n 3
exit $rc
