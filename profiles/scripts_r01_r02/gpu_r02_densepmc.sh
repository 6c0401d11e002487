set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_densepmc
mkdir -p $O
B="python3 bench.py --steps 6 --warmup 2"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || true
python3 - <<'PY' > $O/counters.txt 2>&1 || true
import csv, glob, collections
for d in ("gpurun_out/r02_densepmc/pmc_a", "gpurun_out/r02_densepmc/pmc_b"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:50]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if "dense" in k or "fused" in k or "spmm" in k:
            print(d.split("/")[-1], k, dict(v))
PY
python3 tools/pmc_summary.py --trace $O/trace --pmc $O/pmc_a --top 8 > $O/summary.md 2>&1 || true
echo done
