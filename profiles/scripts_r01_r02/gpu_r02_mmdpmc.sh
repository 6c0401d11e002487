set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_mmdpmc
mkdir -p $O
B="python3 tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 40 --test 20 --eager"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || true
python3 tools/pmc_summary.py --trace $O/trace --pmc $O/pmc_a --top 8 > $O/summary.md 2>&1 || true
python3 - <<'PY' > $O/counters.txt 2>&1 || true
import csv, glob, collections
for d in ("gpurun_out/r02_mmdpmc/pmc_a", "gpurun_out/r02_mmdpmc/pmc_b"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if "mmd" in k or "gen_" in k or "adam" in k:
            print(d.split("/")[-1], k, dict(v))
PY
echo done
