#!/bin/bash
# Round 3: symmetric pred-pred MMD training (mirror slots).  Oracle + bitwise tests,
# the pairwise train/eval step with symmetry on and off, a kernel trace of it, the
# re-pinned example outcomes (the summation order changed), and kernel traces of the
# lin_fwd users (Reddit inference with the wide layer on lin_fwd, GAT products).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_mmd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cgnn_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
B="tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 200 --test 100"
for sym in 1 0 1 0; do
  CGNN_MMD_SYM=$sym timeout -k 10 200 python3 -u $B > $O/pair_sym$sym.log 2>&1 || { echo "bench failed"; tail $O/pair_sym$sym.log; exit 1; }
  echo "sym=$sym $(tail -n 1 $O/pair_sym$sym.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pair_trace -o run -- python3 -u $B --eager --train 40 --test 20 > $O/pair_trace.log 2>&1 || { echo trace failed; tail $O/pair_trace.log; exit 1; }
timeout -k 10 400 python3 -u tools/pin_examples.py $O/expected_examples.json > $O/pin.log 2>&1 || { echo pin failed; tail -20 $O/pin.log; exit 1; }
tail -n 3 $O/pin.log
CGNN_INFER_LIN_KMAX=768 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_trace -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 > $O/reddit_trace.log 2>&1 || { echo trace failed; tail $O/reddit_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gat_trace -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/gat_trace.log 2>&1 || { echo gat trace failed; tail $O/gat_trace.log; exit 1; }
find $O -name "*kernel_trace.csv" -size +4M -delete
python3 - <<'EOF'
import csv, glob
for name in ("pair_trace", "reddit_trace", "gat_trace"):
    f = glob.glob("gpurun_out/r03_mmd/%s/**/*kernel_stats.csv" % name, recursive=True)
    if not f: print(name, "no stats"); continue
    for r in list(csv.DictReader(open(f[0])))[:12]:
        print(name, r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r.get("Percentage", ""))
EOF
echo done
