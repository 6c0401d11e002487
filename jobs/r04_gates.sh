#!/bin/bash
# Round 4: re-pin the three example gates (confounder gate now at the reference's 32 runs)
# and record their outcomes under SETTINGS.compat_scores (reference scoring statistics)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_gates
mkdir -p $O
timeout -k 10 400 python -u tools/pin_examples.py $O/expected_examples.json > $O/pin.log 2>&1 || { echo pin failed; tail -20 $O/pin.log; exit 1; }
tail -n 1 $O/pin.log
timeout -k 10 400 python -u tools/pin_examples.py --compat $O/compat_examples.json > $O/pin_compat.log 2>&1 || { echo compat failed; tail -20 $O/pin_compat.log; exit 1; }
tail -n 1 $O/pin_compat.log
echo done
