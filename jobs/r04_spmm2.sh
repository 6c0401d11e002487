#!/bin/bash
# spmm_ell: unconditional gathers, row scale loaded first; spmm_ce: row data loaded before the gathers (in-tree) vs the column-prefetch commit (sp_v1)
# vs the previous form (sp_v1); headline bench and arxiv, two rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_spmm2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gnn_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for round in 1 2; do
  for v in base sp_v1; do
    lib=""
    [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
    CGNN_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_${v}_$round.log 2>&1 || { echo "bench $v failed"; tail $O/bench_$v.log; exit 1; }
    echo "$v bench $(grep "^{" $O/bench_${v}_$round.log | cut -c90-140)"
    CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv_$v.log 2>&1 || { echo "arxiv $v failed"; exit 1; }
    echo "$v arxiv $(tail -n 1 $O/arxiv_$v.log | cut -c90-150)"
  done
done
