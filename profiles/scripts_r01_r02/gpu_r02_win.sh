#!/bin/bash
# LDS-windowed SpMM: GPU tests, micro-bench on the reordered products shape, and the
# reorder-refinement A/B of the headline epoch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/win
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -k "spmm_win" -x -v --timeout 120 --timeout-method thread \
    > $O/pytest_win.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_win.log; exit 1; }
tail -2 $O/pytest_win.log
timeout -k 10 300 python -u tools/bench_spmm.py --id-order shuffled --reorder --win 64,128,256 --reps 20 \
    > $O/bench_spmm.log 2>&1 || { echo "bench_spmm failed"; tail -20 $O/bench_spmm.log; exit 1; }
cat $O/bench_spmm.log
bash profiles/scripts_r01_r02/gpu_ab_refine.sh ${REFINE:-0 4}
