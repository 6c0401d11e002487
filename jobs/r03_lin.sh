#!/bin/bash
# Round 3: spill-free lin_fwd / lin_bwd_data loaders.  Numerics of every dense-layer
# user (linear, GAT, GCN, SAGE, inference), then GAT products epoch, Reddit inference
# with the wide first layer on lin_fwd vs hipBLASLt, GCN headline bench, and a kernel
# trace of the Reddit run.  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_lin
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_linear_gpu.py tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_$i.log 2>&1 || { echo "gat failed"; tail $O/gat_$i.log; exit 1; }
  echo "gat $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_$i.log)"
done
for k in 768 256; do
  CGNN_INFER_LIN_KMAX=$k timeout -k 10 200 python3 -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_k$k.log 2>&1 || { echo reddit failed; tail $O/reddit_k$k.log; exit 1; }
  echo "reddit kmax=$k $(grep -o '"value": [0-9.]*' $O/reddit_k$k.log)"
done
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
CGNN_INFER_LIN_KMAX=768 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/reddit_trace -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 > $O/reddit_trace.log 2>&1 || { echo trace failed; tail $O/reddit_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gat_trace -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/gat_trace.log 2>&1 || { echo gat trace failed; tail $O/gat_trace.log; exit 1; }
python3 - <<'EOF'
import csv, glob
for name in ("reddit_trace", "gat_trace"):
    f = glob.glob("gpurun_out/r03_lin/%s/**/run_kernel_stats.csv" % name, recursive=True)
    if not f: print(name, "no stats"); continue
    rows = list(csv.DictReader(open(f[0])))
    for r in rows:
        if "lin_" in r["Name"] or "Cijk" in r["Name"]:
            print(name, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
EOF
echo done
