#!/bin/bash
# Round 3: forward AX-tile prefetch (12 waves) A/B; backward with the next tile's Philox
# draw interleaved with the products; GNN GPU tests; kernel trace of both arms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_fwdpf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gnn.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gnn.log | head -20; tail -n 30 $O/pytest_gnn.log; exit 1; }
echo "$(tail -n 1 $O/pytest_gnn.log)"
CGNN_FWD_PREFETCH=1 timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or benched or hipgraph" > $O/pytest_pf.log 2>&1 \
    || { echo "pf tests failed"; grep -E "FAILED|Error|assert" $O/pytest_pf.log | head -20; tail -n 30 $O/pytest_pf.log; exit 1; }
echo "pf $(tail -n 1 $O/pytest_pf.log)"
for v in 0 1 0 1; do
  CGNN_FWD_PREFETCH=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_pf$v.log 2>&1 || { echo bench failed; tail $O/bench_pf$v.log; exit 1; }
  echo "pf=$v $(tail -n 1 $O/bench_pf$v.log | cut -c1-150)"
done
for v in 0 1; do
  CGNN_FWD_PREFETCH=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/prof$v.log 2>&1 || { echo prof failed; tail $O/prof$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in "01":
    f = glob.glob("gpurun_out/r03_fwdpf/prof%s/**/*kernel_stats.csv" % v, recursive=True)
    for r in list(csv.DictReader(open(f[0]))):
        if "gcn_" in r["Name"] or "spmm" in r["Name"] or "adam" in r["Name"] or "slab" in r["Name"]:
            print(v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find $O -name "*_trace.csv" -delete
echo done
