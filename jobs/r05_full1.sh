#!/bin/bash
# Round 5: whole GPU suite after the gather-header / CGNN batching changes, smoke, bench,
# and a kernel trace of the headline epoch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_full1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
tail -n 30 $O/epoch_trace.txt
echo done
