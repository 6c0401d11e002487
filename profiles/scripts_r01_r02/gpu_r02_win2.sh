#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/win2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -k "spmm_win" -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_win.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_win.log; exit 1; }
tail -1 $O/pytest_win.log
timeout -k 10 300 python -u tools/bench_spmm.py --id-order shuffled --reorder --win 256,384,512,256:16,384:16,512:16 --reps 20 \
    > $O/bench_spmm.log 2>&1 || { echo "bench_spmm failed"; tail -20 $O/bench_spmm.log; exit 1; }
grep -E '"ld": 128' $O/bench_spmm.log
export CGNN_SPMM_WIN=0
bash profiles/scripts_r01_r02/gpu_ab_refine.sh 0 4
