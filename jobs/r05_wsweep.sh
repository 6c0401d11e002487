#!/bin/bash
# Round 5: staged CGNN forward / backward over waves per block (1, 2, 4, 8) and every state
# placement, d = 200, H = 20, R = 256, N = 500, at 400 and 736 edges (committed build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_wsweep
mkdir -p $O
for e in 400 736; do
  timeout -k 10 300 python -u tools/ab_staged.py --d 200 --edges $e --R 256 --n 500 --h 20 > $O/sweep_$e.log 2>&1 || { echo sweep $e failed; tail $O/sweep_$e.log; exit 1; }
  grep '^{' $O/sweep_$e.log
done
echo done
