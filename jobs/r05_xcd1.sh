#!/bin/bash
# Round 5: headline A/B of the XCD block remap: contiguous range per XCD (default) vs
# interleaved chunks of 64 / 512 blocks (gnn_sparse.hip rebuilt with CGNN_XCD_CHUNK)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_xcd1
mkdir -p $O
for r in 1 2; do
  for v in base x64 x512; do
    if [ $v = base ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abv/$v/_hip.cpython-310-x86_64-linux-gnu.so; fi
    timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > $O/bench_${v}_$r.log 2>&1 || { echo bench $v failed; tail $O/bench_${v}_$r.log; exit 1; }
    echo $v $r $(tail -n 1 $O/bench_${v}_$r.log | cut -c1-120)
  done
done
for v in base x512; do
  if [ $v = base ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abv/$v/_hip.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o run -- python3 bench.py --steps 10 --warmup 5 > $O/kt_$v.log 2>&1 || { echo trace $v failed; tail $O/kt_$v.log; exit 1; }
  python3 tools/epoch_trace.py $O/kt_$v/run_kernel_trace.csv > $O/epoch_$v.txt 2>&1 || true
done
echo done
