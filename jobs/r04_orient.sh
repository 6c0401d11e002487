#!/bin/bash
# CGNN().orient_directed_graph on RandomGraphGenerator(200) data at the reference settings (time-boxed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_orient
mkdir -p $O
timeout -k 10 480 python -u tools/time_orient.py --seconds 300 > $O/orient.log 2>&1 || { echo orient failed; tail -20 $O/orient.log; exit 1; }
tail -n 2 $O/orient.log
