#!/bin/bash
# Round 5: time the three example gates again (outcomes must match the pinned file)
# (pin_examples writes the outcomes and wall times; tests/data keeps the pinned ones)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_gates
mkdir -p $O
timeout -k 10 400 python -u tools/pin_examples.py $O/expected_examples.json > $O/pin.log 2>&1 || { echo pin failed; tail -20 $O/pin.log; exit 1; }
tail -n 1 $O/pin.log
timeout -k 10 400 python -u tools/pin_examples.py --compat $O/compat_examples.json > $O/pin_compat.log 2>&1 || { echo compat failed; tail -20 $O/pin_compat.log; exit 1; }
tail -n 1 $O/pin_compat.log
echo done
