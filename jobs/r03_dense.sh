#!/bin/bash
# Round 3: GCN dense kernels (bias-initialised accumulators, batched LDS operand reads,
# compile-time dropout switch, double-buffered fused-backward staging) and the
# restored branchy lin_* loaders outside lin_fwd's wide-K variants.  Tests, headline
# bench, kernel traces of the GCN epoch and of GAT products.  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_dense
mkdir -p $O
summ() {   # dir label
  python3 - "$1" "$2" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
if not f: print(sys.argv[2], "no stats"); sys.exit(0)
for r in list(csv.DictReader(open(f[0])))[:14]:
    print(sys.argv[2], r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_gnn_linear_gpu.py tests/test_gat_fused_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$i.log 2>&1 || { echo bench failed; tail $O/bench_$i.log; exit 1; }
  echo "bench $(grep -o '"value": [0-9.]*' $O/bench_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log)"
done
for k in default 256; do
  if [ $k = default ]; then kv=""; else kv=$k; fi
  CGNN_INFER_LIN_KMAX=$kv timeout -k 10 200 python3 -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_$k.log 2>&1 || { echo "reddit $k failed"; tail $O/reddit_$k.log; exit 1; }
  echo "reddit kmax=$k $(grep -o '"value": [0-9.]*' $O/reddit_$k.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_trace -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 > $O/reddit_trace.log 2>&1 || { echo "reddit trace failed"; tail $O/reddit_trace.log; exit 1; }
summ $O/reddit_trace reddit
timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat.log 2>&1 || { echo "gat failed"; tail $O/gat.log; exit 1; }
echo "gat $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gcn_trace -o run -- python3 -u bench.py --steps 10 --warmup 3 > $O/gcn_trace.log 2>&1 || { echo "gcn trace failed"; tail $O/gcn_trace.log; exit 1; }
summ $O/gcn_trace gcn
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gat_trace -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/gat_trace.log 2>&1 || { echo "gat trace failed"; tail $O/gat_trace.log; exit 1; }
summ $O/gat_trace gat | grep lin_
find $O -name "*kernel_trace.csv" -size +2M -delete
echo done
