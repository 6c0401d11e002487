#!/bin/bash
# headline dense forward: D^-1/2 loaded with the rows + prologue loads consumed before the
# tile loop (in-tree) vs the round-4 start (dense_v0) vs + keep stores early and an explicit
# vmcnt(6) (dense_v2); then the GPU dense tests and bench.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dense3
mkdir -p $O
for round in 1 2; do
  for v in base dense_v0 dense_v2; do
    lib=""
    [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
    echo -n "$v " >> $O/ab.log
    CGNN_HIP_LIB=$lib timeout -k 10 120 python -u tools/ab_dense.py --iters 20 2>&1 | grep '{' >> $O/ab.log || { echo "ab $v failed"; exit 1; }
  done
done
cat $O/ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-250
