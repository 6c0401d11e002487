#!/bin/bash
# papers100M 12.5 % shard GAT, same box: every row / train-row layer 2 / + train-neighbour
# layer 1 (6 timed epochs after 2 warm-up).  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/papers3
mkdir -p $O
for v in "allrows:CGNN_L2_ALL_ROWS=1" "l2train:CGNN_L1_TRAIN_NBRS=0" "l1l2:CGNN_L1_TRAIN_NBRS=1"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 6 --warmup 2 > $O/$name.log 2>&1 || { echo "$name failed"; tail -n 20 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"peak_gpu_mem_gib": [0-9.]*' $O/$name.log) $(grep -o '"val_acc": [0-9.]*' $O/$name.log)"
done
echo papers3-done
