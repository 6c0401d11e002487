#!/bin/bash
# Round 6: PMC of the wide-MMD train / eval kernels at the orientation shape (d = 200,
# R = 256, N = 500): what bounds them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mmdpmc
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "mmd_mfma16|gen_bwd_staged|gen_fwd_staged" --output-format csv -d $O/p$i -o run -- python3 -u tools/bench_cgnn_batch.py --d 200 --edges 736 --R 256 --train 6 --test 6 --eager > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for i in (1, 2, 3):
    for f in glob.glob("gpurun_out/r06_mmdpmc/p%d/**/*counter_collection.csv" % i, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:48]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in acc:
    print(k)
    for c in sorted(acc[k]):
        print("   %-28s %16.1f per dispatch" % (c, acc[k][c] / max(1, n[k][c])))
PY
find $O -name "*_trace.csv" -delete
echo done
