#!/bin/bash
# A/B of GAT gather-batch variants (abtmp/<name>/_hip*.so) vs the in-tree build on the
# products-shape fused GAT epoch, PMC counters of the in-tree attention kernels, and the
# wide-CGNN GPU tests.  First failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ab_gat
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -k "gat or inference or gcn_benched" -x -q --timeout 200 \
    --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in intree "$@" intree "$@"; do
  if [ $v = intree ]; then lib=""; else lib=$(ls abtmp/$v/_hip*.so); fi
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/$v.log 2>&1 || { echo "$v failed"; tail $O/$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_epoch": [0-9.]*' $O/$v.log)"
done
B="python3 tools/bench_gat.py --steps 3 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_ANY FETCH_SIZE --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || { echo pmca failed; tail $O/pmca.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || { echo pmcb failed; tail $O/pmcb.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
python3 tools/pmc_summary.py --trace $O/trace --pmc $O/pmc_a $O/pmc_b --top 12 > $O/summary.md 2>&1
cat $O/summary.md
timeout -k 10 600 python -u -m pytest tests/test_cgnn_wide_gpu.py -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_wide.log 2>&1 || { echo "pytest wide failed"; tail -n 40 $O/pytest_wide.log; exit 1; }
tail -n 2 $O/pytest_wide.log
timeout -k 10 300 python3 -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit.log 2>&1 || { echo reddit failed; tail $O/reddit.log; exit 1; }
tail -n 1 $O/reddit.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_trace -o run -- python3 tools/bench_gnn_configs.py --config reddit-infer --steps 20 > $O/reddit_trace.log 2>&1 || { echo reddit trace failed; exit 1; }
python3 tools/pmc_summary.py --trace $O/reddit_trace --top 10 > $O/reddit_summary.md 2>&1
cat $O/reddit_summary.md
echo done
