#!/bin/bash
# Round 3: ELL short-row backward aggregation (CGNN_SPMM_ELL 1 / 0): GNN tests, bench A/B,
# kernel trace; then the 1/8-size epoch timeline (per-rank proxy).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ell
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
echo "$(tail -n 1 $O/pytest.log)"
for v in 1 0 1 0; do
  CGNN_SPMM_ELL=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$v.log 2>&1 || { echo bench failed; tail $O/bench_$v.log; exit 1; }
  echo "ell=$v $(tail -n 1 $O/bench_$v.log | cut -c1-150)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_ell/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0]))):
    if "gcn_" in r["Name"] or "spmm" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us min", round(float(r["MinNs"]) / 1e3, 1))
PY
find $O -name "*_trace.csv" -delete
bash jobs/r03_small.sh
