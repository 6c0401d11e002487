#!/bin/bash
# papers100M GAT, rank 0 of 8 dry run with the locality partition (full scale)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_papers
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.log; done) &
HB=$!
timeout -k 10 1000 python -u tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --steps 3 --warmup 1 --partition locality > $O/dry_locality.log 2>&1
rc=$?
kill $HB
tail -n 3 $O/dry_locality.log
exit $rc
