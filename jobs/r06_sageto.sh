#!/bin/bash
# Round 6: GraphSAGE training step alone (no concurrent sampler) vs the pipelined epoch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sageto
mkdir -p $O
timeout -k 10 400 python -u tools/sage_train_only.py > $O/train_only.log 2>&1 || { echo failed; tail -20 $O/train_only.log; exit 1; }
grep '^{' $O/train_only.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/sage_train_only.py --steps 64 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" -delete
echo done
