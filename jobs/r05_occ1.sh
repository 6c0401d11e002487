set -o pipefail
O=gpurun_out/r05_occ1; mkdir -p $O
V=$PWD/abv/occ8/_hip.cpython-310-x86_64-linux-gnu.so
t() { timeout -k 10 300 "$@"; }
t python -u tools/ab_agg.py --only-ell --iters 30 > $O/ell_default.log 2>&1 &&
CGNN_HIP_LIB=$V t python -u tools/ab_agg.py --only-ell --iters 30 > $O/ell_occ8.log 2>&1 &&
t python -u tools/bench_cgnn_batch.py --d 22 > $O/cgnn22_default.log 2>&1 &&
CGNN_HIP_LIB=$V t python -u tools/bench_cgnn_batch.py --d 22 > $O/cgnn22_occ8.log 2>&1 &&
t python -u tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 > $O/cgnn2_default.log 2>&1 &&
CGNN_HIP_LIB=$V t python -u tools/bench_cgnn_batch.py --d 2 --edges 1 --n 1500 > $O/cgnn2_occ8.log 2>&1 &&
t python -u bench.py --steps 30 --warmup 5 > $O/bench_default.log 2>&1 &&
CGNN_HIP_LIB=$V t python -u bench.py --steps 30 --warmup 5 > $O/bench_occ8.log 2>&1 &&
t python -u bench.py --steps 30 --warmup 5 > $O/bench_default2.log 2>&1 &&
CGNN_HIP_LIB=$V t python -u bench.py --steps 30 --warmup 5 > $O/bench_occ8_2.log 2>&1
