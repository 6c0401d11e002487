#!/bin/bash
# Round 3: every BASELINE config with the current kernels (bit-mode dropout), the Reddit
# aligned-row A/B, GAT products epoch, and a kernel trace of the Reddit replay.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_cfgs
mkdir -p $O
run() { local name=$1; shift; timeout -k 10 600 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail $O/$name.log; exit 1; }; echo "$name $(tail -n 1 $O/$name.log | cut -c1-260)"; }
run arxiv python -u tools/bench_gnn_configs.py --config arxiv-gcn3
run reddit python -u tools/bench_gnn_configs.py --config reddit-infer
CGNN_INFER_ALIGN=1 run reddit_align python -u tools/bench_gnn_configs.py --config reddit-infer
run sage python -u tools/bench_gnn_configs.py --config products-sage3
run gat_products python -u tools/bench_gat.py --steps 10 --warmup 2
run papers_s0125 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 0.125 --steps 3 --warmup 1
CGNN_INFER_ALIGN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_prof -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 --warmup 2 > $O/reddit_prof.log 2>&1 || { echo prof failed; tail $O/reddit_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gat_prof -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/gat_prof.log 2>&1 || { echo prof failed; tail $O/gat_prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
for d in ("reddit_prof", "gat_prof"):
    f = glob.glob("gpurun_out/r03_cfgs/%s/**/*kernel_stats.csv" % d, recursive=True)
    for r in list(csv.DictReader(open(f[0])))[:12]:
        print(d, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
PY
find $O -name "*_trace.csv" -delete
echo done
