#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# k_step phase stamps (libkbengine_stamps.so, -DKB_STAMPS) of several workloads on one box,
# then the production build's bench line of each (same box).
# Usage: gpurun -- 'bash tools/gpu_stamps.sh <tag> [workloads...]'   (default: c3 c5 c2)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-st}; shift
WLS=${*:-c3 c5 c2}
O=gpurun_out/$T; mkdir -p $O
for wl in $WLS; do
  timeout -k 10 200 python3 -u bench.py --stamps --workload $wl --steps 200 --warmup 20 > $O/${wl}_stamps.json 2> $O/${wl}_stamps.err || { tail -5 $O/${wl}_stamps.err; exit 1; }
done
for wl in $WLS; do
  timeout -k 10 200 python3 -u bench.py --workload $wl --steps 200 --warmup 20 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
done
python3 tools/show_r05.py $O
