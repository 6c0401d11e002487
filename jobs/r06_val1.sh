#!/bin/bash
# Round 6 validation: whole GPU suite, smoke, multi-rank host/GPU probe + epoch trace, bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_val1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u tools/multirank_host.py > $O/host_gpu.log 2>&1 || { echo host probe failed; tail $O/host_gpu.log; exit 1; }
grep '^{' $O/host_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/multirank_host.py --forms collectives --epochs 10 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_kernels.py $O/prof/run_kernel_trace.csv 8 > $O/epoch_kernels.txt 2>&1 || true
cat $O/epoch_kernels.txt
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
echo done
