#!/bin/bash
# Round 5 late validation after the ELL occupancy cap and the staged-backward changes: the
# whole GPU test suite, smoke, the headline bench (twice), arxiv and the CGNN d = 200 batch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_validate2
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
for k in 1 2; do
timeout -k 10 300 python -u bench.py > $O/bench_$k.log 2>&1 || { echo bench failed; tail $O/bench_$k.log; exit 1; }
grep '^{' $O/bench_$k.log | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_gnn_configs.py --config arxiv-gcn3 > $O/arxiv.log 2>&1 || { echo arxiv failed; tail $O/arxiv.log; exit 1; }
tail -n 1 $O/arxiv.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_cgnn_batch.py --d 200 --edges 400 --R 256 --n 500 --h 20 > $O/cgnn_d200.log 2>&1 || { echo cgnn failed; tail $O/cgnn_d200.log; exit 1; }
grep '^{' $O/cgnn_d200.log | cut -c1-250
echo done
