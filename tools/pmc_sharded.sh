#!/bin/bash
# PMC passes of the world-1 sharded round (bench.py --sharded: k_scansum + k_step, then the
# plain plan's k_pair) per workload, FETCH_SIZE then WRITE_SIZE in separate kernel-trace runs,
# into gpurun_out/pmc_traffic.json under "<workload>_sharded" (dist.bench_main's traffic).
# Usage: tools/pmc_sharded.sh GIT_HEAD [WORKLOADS...]   (default c3 c5)
HEAD=${1:?git head}; shift
WLS=${*:-c3 c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for wl in $WLS; do
  steps=100; [ "$wl" = "c5" ] && steps=60
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 5 -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmcs_${wl}_$grp -o run \
        -- python3 bench.py --sharded --workload $wl --steps $steps --warmup 5 \
        > gpurun_out/pmcs_${wl}_$grp.log 2>&1 || exit $?
  done
  python3 tools/pmc_summarise.py pmcs_$wl gpurun_out/pmc_traffic.json ${wl}_sharded $HEAD || exit $?
done
exit 0
