#!/bin/bash
# Round 5: the reference-settings orientation run after the no-Gm backward (full run),
# and a 30-second kernel-traced slice of it (where a batch's time goes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_orient3
mkdir -p $O
timeout -k 10 400 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail $O/orient.log; exit 1; }
tail -n 1 $O/orient.log | cut -c1-400
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/time_orient.py --seconds 30 > $O/orient_prof.log 2>&1 || { echo prof failed; tail $O/orient_prof.log; exit 1; }
echo done
