#!/bin/bash
# Train-row layer 2 in the fused GAT (GPU tests + products epoch with / without it),
# then the headline A/B (packed layer-2 rows, hipGraph replay).  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/l2gat
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gat_fused_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gat.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest_gat.log; exit 1; }
tail -n 2 $O/pytest_gat.log
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_products.log 2>&1 || { echo "gat failed"; tail -n 20 $O/gat_products.log; exit 1; }
echo "gat $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_products.log) $(grep -o '"train_loss": [0-9.]*' $O/gat_products.log) $(grep -o '"val_acc": [0-9.]*' $O/gat_products.log)"
CGNN_L2_ALL_ROWS=1 timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_products_allrows.log 2>&1 || { echo "gat allrows failed"; exit 1; }
echo "gat-allrows $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_products_allrows.log) $(grep -o '"train_loss": [0-9.]*' $O/gat_products_allrows.log) $(grep -o '"val_acc": [0-9.]*' $O/gat_products_allrows.log)"
bash profiles/scripts_r01_r02/gpu_r02_ab2.sh
