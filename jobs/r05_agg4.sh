#!/bin/bash
# Round 5: block-cooperative chunks in the fused aggregation (narrow row window)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_agg4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "agg_fwd or fused_aggregation or benched_config" > $O/pytest.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 200 python -u tools/ab_agg.py > $O/ab_default.log 2>&1 || { echo ab failed; tail $O/ab_default.log; exit 1; }
tail -n 1 $O/ab_default.log
for v in v_rpc2 v_g1 v_g2; do
  CGNN_HIP_LIB=$PWD/abtmp/_hip_$v.so timeout -k 10 200 python -u tools/ab_agg.py --only-agg > $O/ab_$v.log 2>&1 || { echo ab $v failed; tail $O/ab_$v.log; exit 1; }
  tail -n 1 $O/ab_$v.log
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex "gcn_agg" --output-format csv -d $O/pmc -o run -- python3 tools/ab_agg.py --iters 2 --only-agg > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
echo done
