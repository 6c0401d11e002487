set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_misc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_gnn_configs.py --config reddit-infer > $O/reddit.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gnn_configs.py --config reddit-infer --reorder none > $O/reddit_noreorder.log 2>&1 || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/bench_gnn_configs.py --config products-sage3 --steps 1 --warmup 1 --shared-gpu > $O/sage_dp2_shared.log 2>&1 || exit 1
echo done
