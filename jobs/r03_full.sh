#!/bin/bash
# Round 3 validation: the whole GPU test suite, smoke, the headline bench, and the
# full-size papers100M rank-0-of-8 dry run with the communication-free layer 1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_full4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
tail -n 1 $O/bench.log
timeout -k 10 900 python -u tools/bench_gnn_configs.py --config papers-gat2 --scale 1.0 --steps 3 --warmup 1 --emulate-world 8 > $O/gat_emulate_r0of8_full.log 2>&1 || { echo emulate failed; tail $O/gat_emulate_r0of8_full.log; exit 1; }
tail -n 1 $O/gat_emulate_r0of8_full.log
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo arxiv failed; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_products.log 2>&1 || { echo gat failed; tail $O/gat_products.log; exit 1; }
tail -n 1 $O/gat_products.log
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit.log 2>&1 || { echo reddit failed; tail $O/reddit.log; exit 1; }
tail -n 1 $O/reddit.log
echo done
