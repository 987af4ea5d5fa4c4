#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# PMC passes for the roofline's `traffic` (MI355X_MICROARCH.md HBM section): per workload
# one rocprofv3 run per counter (FETCH_SIZE, then WRITE_SIZE; kernel trace only, never
# with a runtime / sys trace), each under its own hard time limit.
# Usage: tools/pmc_r04.sh GIT_HEAD [WORKLOADS...]   (default c3 c5)
HEAD=${1:?git head}; shift
WLS=${*:-c3 c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
for wl in $WLS; do
  steps=200; [ "$wl" = "c5" ] && steps=100
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 5 -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_${wl}_$grp -o run \
        -- python3 bench.py --workload $wl --steps $steps --warmup 5 --no-cpu-baseline --no-secondary \
        > gpurun_out/pmc_${wl}_$grp.log 2>&1 || exit $?
  done
  python3 tools/pmc_summarise.py pmc_$wl gpurun_out/pmc_traffic.json $wl $HEAD || exit $?
done
exit 0
