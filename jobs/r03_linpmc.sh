#!/bin/bash
# lin_fwd / lin_bwd_data at SAGE layer-0 shapes (200 K rows): kernel trace + two PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_linpmc
mkdir -p $O
B="python3 tools/bench_lin.py --reps 3 --rows 200000"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_ANY FETCH_SIZE --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || { echo pmca failed; tail $O/pmca.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR WRITE_SIZE --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || { echo pmcb failed; tail $O/pmcb.log; exit 1; }
python3 tools/pmc_summary.py --trace $O/trace --pmc $O/pmc_a $O/pmc_b --top 12 > $O/summary.md 2>&1
python3 - > $O/raw.txt <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for d in ("pmc_a", "pmc_b"):
    for f in glob.glob("gpurun_out/r03_linpmc/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:48]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    if "lin_" in k:
        print(k, {c: round(x) for c, x in sorted(v.items())})
PY
find $O -name "*_trace.csv" -size +3M -delete
echo done
