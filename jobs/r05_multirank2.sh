#!/bin/bash
# Round 5: 2-rank --shared-gpu papers-gat2 rehearsal at scale 0.1 (the
# partition is computed by rank 0 only and broadcast; per-rank setup seconds reported)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_multirank2
mkdir -p $O
( while sleep 20; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
   tools/bench_gnn_configs.py --config papers-gat2 --scale 0.1 --shared-gpu --steps 3 --warmup 1 > $O/papers_rehearsal.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { echo rehearsal failed $rc; grep -v "^\[W" $O/papers_rehearsal.log | tail -n 30; exit 1; }
grep 'bench_gnn_configs rank' $O/papers_rehearsal.log
grep '^{' $O/papers_rehearsal.log | cut -c1-700
echo done
