#!/bin/bash
# Round 3: spmm_ce long rows on a whole wave (train rows ordered long-first), aligned
# Reddit inference rows by default: GNN GPU tests, headline bench, arxiv + Reddit configs,
# kernel trace of the headline epoch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ce
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_gat_fused_gpu.py tests/test_gnn_linear_gpu.py tests/test_rccl_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gnn.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gnn.log | head -20; tail -n 30 $O/pytest_gnn.log; exit 1; }
echo "$(tail -n 1 $O/pytest_gnn.log)"
run() { local name=$1; shift; timeout -k 10 600 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail $O/$name.log; exit 1; }; echo "$name $(tail -n 1 $O/$name.log | cut -c1-200)"; }
run bench1 python -u bench.py --steps 40 --warmup 5
run bench2 python -u bench.py --steps 40 --warmup 5
run arxiv python -u tools/bench_gnn_configs.py --config arxiv-gcn3
run reddit python -u tools/bench_gnn_configs.py --config reddit-infer
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03_ce/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0]))):
    if "gcn_" in r["Name"] or "spmm" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us min", round(float(r["MinNs"]) / 1e3, 1))
PY
find $O -name "*_trace.csv" -delete
echo done
