#!/bin/bash
# Round 5: graph-captured sampler, ablated (graph x publish), then the SAGE bench + trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_sage3
mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py -x -v --timeout 120 --timeout-method thread -k "pipelined_sampler_matches_device" > $O/ablate.log 2>&1 \
    || { echo "ablation failed"; grep -E "PASSED|FAILED|Error|assert" $O/ablate.log | head -30; exit 1; }
grep -c PASSED $O/ablate.log
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py tests/test_gnn_gpu.py -x -q --timeout 120 --timeout-method thread -k "sage or sampler" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage_$r.log 2>&1 || { echo sage failed; tail $O/sage_$r.log; exit 1; }
tail -n 1 $O/sage_$r.log | cut -c1-250
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo done
