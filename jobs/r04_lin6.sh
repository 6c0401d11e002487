#!/bin/bash
# weight-stationary kernels: PMC at the arxiv shapes; stores-first variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lin6
mkdir -p $O
for v in base stfirst; do
  lib=""
  [ $v != base ] && lib=$PWD/abtmp/$v/_hip.cpython-310-x86_64-linux-gnu.so
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_lin.py --shape arxiv --reps 10 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail $O/kt_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/kt_$v.log)"
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES SQ_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 tools/bench_lin.py --shape arxiv --reps 2 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for i in (1, 2, 3):
    for f in glob.glob("gpurun_out/r04_lin6/p%d/**/*counter_collection.csv" % i, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "lin_ws" not in k: continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[(k, i)].add(r["Dispatch_Id"])
for k in acc:
    n = max(len(nd[(k, i)]) for i in (1, 2, 3))
    print(k, "dispatches", n)
    for c in sorted(acc[k]):
        print("   %-24s %.4g" % (c, acc[k][c] / max(1, len(nd[(k, 1)]) if c in ("SQ_WAVES",) else n)))
PY
find $O -name "*_trace.csv" -delete
