#!/bin/bash
# Round 6: pipelined persistent ELL aggregation (CGNN_ELL_FORM=1) vs the one-shot kernel (0):
# tests, interleaved headline benches, and a kernel trace of the new form
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ell1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gnn_gpu.py tests/test_cgnn_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "ell or benched_config or fused_backward or verbose" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
for f in 0 1; do
CGNN_ELL_FORM=$f timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > $O/bench_f${f}_$r.log 2>&1 || { echo bench failed; tail $O/bench_f${f}_$r.log; exit 1; }
echo "form $f run $r: $(grep '^{' $O/bench_f${f}_$r.log | cut -c1-160)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
python3 tools/epoch_trace.py $O/prof/run_kernel_trace.csv 4 > $O/epoch_trace.txt 2>&1 || true
cat $O/epoch_trace.txt
echo done
