#!/bin/bash
# Round 5 validation: the whole GPU test suite, smoke, the headline bench, the GNN
# configs (arxiv, SAGE with a kernel trace, GAT products, Reddit inference) and the
# full-size papers100M rank-0-of-8 dry run with the locality partition
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${VAL_OUT:-r05_validate}
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo arxiv failed; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config products-sage3 > $O/sage.log 2>&1 || { echo sage failed; tail $O/sage.log; exit 1; }
tail -n 1 $O/sage.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sage_kt -o run -- python3 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 > $O/sage_kt.log 2>&1 || { echo sage kt failed; tail $O/sage_kt.log; exit 1; }
timeout -k 10 300 python -u tools/bench_gat.py --steps 10 --warmup 2 > $O/gat_products.log 2>&1 || { echo gat failed; tail $O/gat_products.log; exit 1; }
tail -n 1 $O/gat_products.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit.log 2>&1 || { echo reddit failed; tail $O/reddit.log; exit 1; }
tail -n 1 $O/reddit.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 256 --n 500 --h 20 > $O/cgnn_d200.log 2>&1 || { echo cgnn failed; tail $O/cgnn_d200.log; exit 1; }
grep '^{' $O/cgnn_d200.log | cut -c1-250
timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 32 --n 500 --h 20 --train 20 --test 10 --fast > $O/cgnn_d200_fast.log 2>&1 || { echo cgnn fast failed; tail $O/cgnn_d200_fast.log; exit 1; }
grep '^{' $O/cgnn_d200_fast.log | cut -c1-250
timeout -k 10 1000 python -u tools/bench_gnn_configs.py --config papers-gat2 --emulate-world 8 --emulate-rank 0 --partition locality --steps 10 --warmup 2 > $O/papers_dry_r0of8.log 2>&1 || { echo papers failed; tail $O/papers_dry_r0of8.log; exit 1; }
tail -n 1 $O/papers_dry_r0of8.log | cut -c1-300
find $O -name "*_trace.csv" -delete
echo done
