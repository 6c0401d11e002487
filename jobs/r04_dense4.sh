#!/bin/bash
# headline dense forward: packed bf16 epilogue (in-tree) vs HEAD (sp_v1): kernel A/B, the GPU
# GNN tests, bench.py A/B two rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dense4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for round in 1 2; do
  for v in base sp_v1; do
    lib=""
    [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
    echo -n "$v " >> $O/ab.log
    CGNN_HIP_LIB=$lib timeout -k 10 120 python -u tools/ab_dense.py --iters 20 2>&1 | grep '{' >> $O/ab.log || { echo "ab $v failed"; exit 1; }
    CGNN_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_${v}_$round.log 2>&1 || { echo "bench $v failed"; exit 1; }
    echo "$v $(grep '^{' $O/bench_${v}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cat $O/ab.log
