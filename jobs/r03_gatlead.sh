#!/bin/bash
# Round 3: GAT per-head score loads by the group leader + DPP broadcast (CGNN_GAT_LEAD 1 / 0):
# GAT GPU tests, products epoch A/B, papers 12.5 % shard, kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_gatlead
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gat_fused_gpu.py tests/test_gnn_gpu.py -k "gat" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
echo "$(tail -n 1 $O/pytest.log)"
for v in 1 0 1; do
  CGNN_GAT_LEAD=$v timeout -k 10 300 python -u tools/bench_gat.py --steps 8 --warmup 2 > $O/gat_$v.log 2>&1 || { echo bench failed; tail $O/gat_$v.log; exit 1; }
  echo "lead=$v $(tail -n 1 $O/gat_$v.log | cut -c1-160)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_gatlead/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0]))):
    if "gat_" in r["Name"]:
        print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find $O -name "*_trace.csv" -delete
echo done
