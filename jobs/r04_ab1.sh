#!/bin/bash
# A/B of fused dense backward forms (tools/ab_dense.py, products shape, random operands)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_ab1
mkdir -p $O
for round in 1 2; do
  for v in v1 default v3 v5; do
    if [ $v = default ]; then unset CGNN_HIP_LIB; else export CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so; fi
    timeout -k 10 120 python -u tools/ab_dense.py --iters 20 >> $O/ab.log 2>&1 || { echo "ab $v failed"; tail $O/ab.log; exit 1; }
  done
done
unset CGNN_HIP_LIB
cat $O/ab.log | grep '{'
export CGNN_HIP_LIB=$PWD/abtmp/_hip_v5.so
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU --kernel-include-regex "gcn_" --output-format csv -d $O/pmc_a -o run -- python3 tools/ab_dense.py --iters 3 > $O/pmca.log 2>&1 || { echo pmc_a failed; tail $O/pmca.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "gcn_" --output-format csv -d $O/pmc_b -o run -- python3 tools/ab_dense.py --iters 3 > $O/pmcb.log 2>&1 || { echo pmc_b failed; tail $O/pmcb.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("pmc_a", "pmc_b"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob("gpurun_out/r04_ab1/" + d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(d, k, {a: "%.4g" % b for a, b in v.items()})
PY
echo done
