#!/bin/bash
# Round 6: CGNN orientation at the reference settings on the committed tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_final4
mkdir -p $O
timeout -k 10 600 python -u tools/time_orient.py > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 5 $O/orient.log
echo done
