#!/bin/bash
# Round 5: where a 1/8-size GCN epoch's 0.8 ms goes (one rank's share at 8 GPUs): kernel
# traces of the one-GPU path and the collectives path on the scale-1/8 products graph
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_eighth1
mkdir -p $O
for f in one_gpu_captured collectives; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$f -o run -- python3 tools/multirank_host.py --forms $f --epochs 20 > $O/$f.log 2>&1 || { echo $f failed; tail $O/$f.log; exit 1; }
  grep '^{' $O/$f.log
done
echo done
