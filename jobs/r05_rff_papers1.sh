#!/bin/bash
# Round 5: Fourier-feature MMD narrow vs wide form by D; papers100M rank-0-of-8 dry run
# with a kernel trace (where the 75 ms epoch goes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_rff_papers1
mkdir -p $O
timeout -k 10 300 python -u tools/ab_rff.py > $O/ab_rff.log 2>&1 || { echo ab_rff failed; tail $O/ab_rff.log; exit 1; }
grep '^{' $O/ab_rff.log
( while sleep 20; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --partition locality --steps 5 --warmup 2 > $O/papers_dry.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { echo papers failed $rc; tail -n 20 $O/papers_dry.log; exit 1; }
grep 'bench_gnn_configs rank' $O/papers_dry.log
grep '^{' $O/papers_dry.log | cut -c1-400
echo done
