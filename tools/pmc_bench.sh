#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# PMC passes over a short bench run (one counter group per rocprofv3 run, kernel
# trace only): FETCH_SIZE and WRITE_SIZE per dispatch of every kernel.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-pmcb}
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 5 -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/${TAG}_$grp -o run \
      -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_$grp.log 2>&1 || exit $?
done
exit 0
