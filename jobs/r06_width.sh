#!/bin/bash
# Round 6: layer-1 SpMM time against gathered width / pitch on the headline graph
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_width
mkdir -p $O
timeout -k 10 400 python -u tools/bench_spmm_width.py > $O/width.log 2>&1 || { echo width failed; tail $O/width.log; exit 1; }
cat $O/width.log
echo done
