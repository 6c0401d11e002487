#!/bin/bash
# A/B of SpMM kernel variants (abtmp/<name>/_hip*.so) against the in-tree build: the
# micro-bench on the reordered products shape and the headline epoch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_spmm
mkdir -p $O
for v in intree "$@" intree "$@"; do
  if [ $v = intree ]; then lib=""; else lib=$(ls abtmp/$v/_hip*.so); fi
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_spmm.py --id-order shuffled --reorder --reps 20 > $O/spmm_$v.log 2>&1 || exit 1
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > $O/bench_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' $O/bench_$v.log) | $(grep '"ld": 128\|"ld": 64\|spmm_ce' $O/spmm_$v.log | grep -o '"ms": [0-9.]*' | tr '\n' ' ')"
done
# multi-rank HIP path on one GPU (gloo): 1 vs 2 vs 4 ranks, same loss
for w in 1 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $w --shared-gpu --steps 5 --warmup 2 > $O/rehearse$w.log 2>&1 || { echo "rehearsal $w failed"; tail -20 $O/rehearse$w.log; exit 1; }
  echo "ranks=$w $(grep -o '"train_loss": [0-9.]*' $O/rehearse$w.log) $(grep -o '"val_acc": [0-9.]*' $O/rehearse$w.log)"
done
