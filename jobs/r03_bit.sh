#!/bin/bash
# Round 3: bit-mode dropout (p = 1/2: one Philox draw per row and half for all 8 hidden
# blocks) in every GNN kernel -- GNN GPU tests, bench A/B of the fused backward forms,
# kernel trace + PMC of the dense kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_bit2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_gpu.py tests/test_gat_fused_gpu.py tests/test_gnn_linear_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gnn.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gnn.log | head -20; tail -n 30 $O/pytest_gnn.log; exit 1; }
echo "$(tail -n 1 $O/pytest_gnn.log)"
for v in tb1 v1 tb1 v1; do
  case $v in tb2) E="CGNN_FUSED_BWD_TB=2";; tb1) E="CGNN_FUSED_BWD_TB=1";; v1) E="CGNN_FUSED_BWD_V1=1";; esac
  env $E timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench_$v.log 2>&1 || { echo bench failed; tail $O/bench_$v.log; exit 1; }
  echo "$v $(tail -n 1 $O/bench_$v.log | cut -c1-150)"
done
B="python3 -u bench.py --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $B > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU --kernel-include-regex "gcn_" --output-format csv -d $O/pmc_a -o run -- $B > $O/pmca.log 2>&1 || { echo pmc_a failed; tail $O/pmca.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "gcn_" --output-format csv -d $O/pmc_b -o run -- $B > $O/pmcb.log 2>&1 || { echo pmc_b failed; tail $O/pmcb.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r03_bit2/prof/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
for d in ("pmc_a", "pmc_b"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob("gpurun_out/r03_bit2/" + d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(d, k, {a: "%.4g" % b for a, b in v.items()})
PY
find $O -name "*_trace.csv" -delete
echo done
