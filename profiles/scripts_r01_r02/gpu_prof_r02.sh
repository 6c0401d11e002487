set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02prof
mkdir -p $O
B="python3 bench.py --steps 10 --warmup 3"
for v in reo:--reorder=lp-cm noreo:--reorder=none; do
  tag=${v%%:*}; arg=${v#*:}
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/trace -o run -- $B $arg > $O/$tag.trace.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/$tag/pmc_a -o run -- $B $arg > $O/$tag.pmca.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$tag/pmc_b -o run -- $B $arg > $O/$tag.pmcb.log 2>&1 || exit 1
done
echo profdone
