#!/bin/bash
# Round 5: short-row SpMM without the XCD remap (init rows spread over all XCDs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_sage7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 120 --timeout-method thread -k "short_rows" > $O/short.log 2>&1 \
    || { echo "short tests failed"; grep -E "FAILED|Error|assert" $O/short.log | head -20; tail -n 30 $O/short.log; exit 1; }
tail -n 1 $O/short.log
timeout -k 10 300 python -u tools/ab_short.py > $O/ab.log 2>&1 || { echo ab failed; tail $O/ab.log; exit 1; }
tail -n 2 $O/ab.log | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py tests/test_gnn_gpu.py -x -q --timeout 120 --timeout-method thread -k "sage or sampler or spmm" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
tail -n 1 $O/sage_$r.log | cut -c1-250
done
timeout -k 10 300 python -u tools/sage_host.py > $O/host.log 2>&1 || { echo host probe failed; tail $O/host.log; exit 1; }
tail -n 2 $O/host.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo done
