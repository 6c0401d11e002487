#!/bin/bash
# PMC of the staged backward (d = 200, H = 20, R = 256, W = 4, state in global memory)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_stpmc
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 -u tools/ab_staged.py --h 20 --reps 3 --only bwd:4:2 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for i in (1, 2):
    f = glob.glob("gpurun_out/r04_stpmc/p%d/**/*counter_collection.csv" % i, recursive=True)
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "gen_bwd_staged" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    for k in sorted(acc):
        print(k, acc[k] / max(1, n[k] // 1), "(sum over %d rows)" % n[k])
PY
find $O -name "*_trace.csv" -delete
echo done
