#!/bin/bash
# Round 3: where a 1/8-size epoch (the per-rank compute of an 8-rank run) spends its time:
# kernel trace with timestamps, one epoch's timeline (kernels and the gaps between them).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_small
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 -u bench.py --steps 20 --warmup 5 --scale 0.125 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 - <<'PY' > $O/timeline.txt
import csv, glob
f = glob.glob("gpurun_out/r03_small/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# epochs: each starts with the layer-1 spmm (spmm_kernel<16...) after warm-up; take the last 3
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void spmm_kernel<16")]
print("layer-1 spmm launches:", len(idx))
for a, b in zip(idx[-4:-1], idx[-3:]):
    t0 = int(rows[a]["Start_Timestamp"])
    print("---- epoch: %.1f us" % ((int(rows[b]["Start_Timestamp"]) - t0) / 1e3))
    prev_end = t0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%8.1f %8.1f gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3, r["Kernel_Name"][:70]))
        prev_end = max(prev_end, e)
PY
head -80 $O/timeline.txt
find $O -name "*_trace.csv" -size +2M -delete
echo done
