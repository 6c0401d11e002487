#!/bin/bash
# GAT layer 1 at the train-neighbour rows in training: GPU tests, products and papers
# 12.5 % shard epochs with / without it.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gatl1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gat_fused_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_gat.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest_gat.log; exit 1; }
tail -n 2 $O/pytest_gat.log
for v in "nbrs:1" "all:0"; do
  name=${v%%:*}; val=${v#*:}
  CGNN_L1_TRAIN_NBRS=$val timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_products_$name.log 2>&1 || { echo "gat $name failed"; tail -n 20 $O/gat_products_$name.log; exit 1; }
  echo "products $name $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_products_$name.log) $(grep -o '"train_loss": [0-9.]*' $O/gat_products_$name.log) $(grep -o '"val_acc": [0-9.]*' $O/gat_products_$name.log)"
done
for v in "nbrs:1" "all:0"; do
  name=${v%%:*}; val=${v#*:}
  CGNN_L1_TRAIN_NBRS=$val timeout -k 10 400 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1 > $O/gat_papers_s0125_$name.log 2>&1 || { echo "papers $name failed"; tail -n 20 $O/gat_papers_s0125_$name.log; exit 1; }
  echo "papers $name $(grep -o '"ms_per_step": [0-9.]*' $O/gat_papers_s0125_$name.log) $(grep -o '"peak_gpu_mem_gib": [0-9.]*' $O/gat_papers_s0125_$name.log) $(grep -o '"val_acc": [0-9.]*' $O/gat_papers_s0125_$name.log)"
done
echo gatl1-done
