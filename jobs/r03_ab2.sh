#!/bin/bash
# Round 3, second batch: GAT gather-batch A/B (in-tree EC=2 vs abtmp variants), Reddit
# inference with / without the wide layer on lin_fwd, the pinned example outcomes,
# papers100M 12.5 % shard epoch, long-N public-API timing.  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ab2
mkdir -p $O
for v in intree "$@" intree "$@"; do
  if [ $v = intree ]; then lib=""; else lib=$(ls abtmp/$v/_hip*.so); fi
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_$v.log 2>&1 || { echo "$v failed"; tail $O/gat_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_$v.log)"
done
for k in 768 256; do
  CGNN_INFER_LIN_KMAX=$k timeout -k 10 200 python3 -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_k$k.log 2>&1 || { echo reddit failed; tail $O/reddit_k$k.log; exit 1; }
  echo "reddit kmax=$k $(grep -o '"value": [0-9.]*' $O/reddit_k$k.log)"
done
timeout -k 10 300 python3 -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 > $O/papers_s0125.log 2>&1 || { echo papers failed; tail $O/papers_s0125.log; exit 1; }
tail -n 1 $O/papers_s0125.log
timeout -k 10 300 python3 -u tools/bench_long_n.py --api --N 100000 --train 20 --test 10 > $O/long_api.log 2>&1 || { echo long api failed; tail $O/long_api.log; exit 1; }
tail -n 1 $O/long_api.log
timeout -k 10 400 python3 -u tools/pin_examples.py $O/expected_examples.json > $O/pin.log 2>&1 || { echo pin failed; tail -20 $O/pin.log; exit 1; }
tail -n 1 $O/pin.log
echo done
