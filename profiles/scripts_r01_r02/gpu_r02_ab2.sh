#!/bin/bash
# A/B of the headline after the train-row layer 2: default, packed layer-2 rows
# (--rows mixed), hipGraph replay (--capture).  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2
mkdir -p $O
for v in "default:" "mixed:--rows mixed" "capture:--capture" "mixcap:--rows mixed --capture"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 $args > $O/$name.log 2>&1 || { echo "$name failed"; tail -n 20 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"train_loss": [0-9.]*' $O/$name.log)"
done
echo ab2-done
