#!/bin/bash
# Round 6: CGNN orientation at the reference settings with 512 models per device batch (16 candidates) vs 256
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_orientbm
mkdir -p $O
timeout -k 10 560 python -u tools/time_orient.py --batch-models 512 > $O/orient_512.log 2>&1 || { echo orient failed; tail $O/orient_512.log; exit 1; }
tail -n 1 $O/orient_512.log
echo done
