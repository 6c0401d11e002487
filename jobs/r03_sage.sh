#!/bin/bash
# Round 3: where the SAGE mini-batch pipeline's copyBuffer calls come from -- kernel +
# HIP API trace of a short products-sage3 run (no counters), summarised by API call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sage
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/trace -o run -- python3 -u tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
d = "gpurun_out/r03_sage/trace"
for pat in ("*hip_api_stats.csv", "*kernel_stats.csv"):
    f = glob.glob(d + "/**/" + pat, recursive=True)
    if not f: print("no", pat); continue
    for r in list(csv.DictReader(open(f[0])))[:25]:
        print(pat[1:9], r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
f = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)
if f:
    rows = list(csv.DictReader(open(f[0])))
    print(rows[0].keys())
    c = collections.Counter()
    for r in rows:
        if "Memcpy" in r["Function"] or "Memset" in r["Function"]:
            c[(r["Function"], r.get("Args", "")[:80])] += 1
    for k, v in c.most_common(20): print(v, k)
PY
find $O -name "*_trace.csv" -size +3M -delete
echo done
