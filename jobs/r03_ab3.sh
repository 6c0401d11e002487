#!/bin/bash
# Round 3: (1) lin_* loaders A/B -- in-tree branch-free vs the previous branchy
# variant (abtmp/lin_old) -- via kernel traces of GAT products and Reddit inference;
# (2) PMC of the pairwise MMD train kernel with and without pred-pred symmetry;
# (3) kernel trace of the headline GCN epoch.  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ab3
mkdir -p $O
summ() {   # dir label
  python3 - "$1" "$2" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
if not f: print(sys.argv[2], "no stats"); sys.exit(0)
for r in list(csv.DictReader(open(f[0])))[:14]:
    print(sys.argv[2], r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1))
EOF
}
for v in intree lin_old; do
  if [ $v = intree ]; then lib=""; else lib=$(ls abtmp/$v/_hip*.so); fi
  CGNN_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_$v.log 2>&1 || { echo "gat $v failed"; tail $O/gat_$v.log; exit 1; }
  echo "gat $v $(grep -o '"ms_per_epoch": [0-9.]*' $O/gat_$v.log)"
  CGNN_HIP_LIB=$lib CGNN_INFER_LIN_KMAX=768 timeout -k 10 200 python3 -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit_$v.log 2>&1 || { echo "reddit $v failed"; tail $O/reddit_$v.log; exit 1; }
  echo "reddit768 $v $(grep -o '"value": [0-9.]*' $O/reddit_$v.log)"
  CGNN_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gat_trace_$v -o run -- python3 -u tools/bench_gat.py --steps 4 --warmup 1 > $O/gat_trace_$v.log 2>&1 || { echo "gat trace $v failed"; tail $O/gat_trace_$v.log; exit 1; }
  summ $O/gat_trace_$v gat_$v | grep lin_
  CGNN_HIP_LIB=$lib CGNN_INFER_LIN_KMAX=768 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/reddit_trace_$v -o run -- python3 -u tools/bench_gnn_configs.py --config reddit-infer --steps 20 > $O/reddit_trace_$v.log 2>&1 || { echo "reddit trace $v failed"; exit 1; }
  summ $O/reddit_trace_$v reddit_$v | grep lin_
done
B="tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 --R 320 --h 30 --train 40 --test 20 --eager"
for sym in 1 0; do
  CGNN_MMD_SYM=$sym timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/mmd_pmc_$sym -o run -- python3 $B > $O/mmd_pmc_$sym.log 2>&1 || { echo "pmc $sym failed"; tail $O/mmd_pmc_$sym.log; exit 1; }
done
python3 - <<'EOF'
import csv, glob, collections
for sym in ("1", "0"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in glob.glob("gpurun_out/r03_ab3/mmd_pmc_%s/**/*counter_collection.csv" % sym, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:40]
            if "mmd_rbf" not in k: continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print("sym=" + sym, k, {c: "%.3g" % x for c, x in sorted(v.items())})
EOF
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gcn_trace -o run -- python3 -u bench.py --steps 10 --warmup 3 > $O/gcn_trace.log 2>&1 || { echo "gcn trace failed"; tail $O/gcn_trace.log; exit 1; }
summ $O/gcn_trace gcn
find $O -name "*kernel_trace.csv" -size +2M -delete
echo done
