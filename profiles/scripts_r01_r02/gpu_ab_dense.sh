#!/bin/bash
# A/B of fused dense kernel variants (abtmp/<name>/_hip*.so) against the in-tree build
# on the ogbn-products shape with the headline row pitches.
set -e
mkdir -p gpurun_out/ab_dense
out=gpurun_out/ab_dense/results.log
: > $out
echo "== in-tree" >> $out
timeout -k 10 120 python tools/bench_dense.py --aligned --p 0.5 --reps 30 >> $out 2>&1
for v in "$@"; do
  echo "== $v" >> $out
  CGNN_HIP_LIB=$(ls abtmp/$v/_hip*.so) timeout -k 10 120 python tools/bench_dense.py --aligned --p 0.5 --reps 30 >> $out 2>&1
done
