#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Diagnostic A/B of k_step variants on the c3 bench: each argument is NAME=LIB[:ENV=VAL,...]
# (LIB relative to kafkabalancer_amd/lib; "-" = the production build).  Prints ms/step and
# the per-step kernel times of each variant.  Plans of ablation builds are wrong by design.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/exp; mkdir -p $O
STEPS=${STEPS:-1000}
WL=${WL:-c3}
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*:}
  [ "$lib" = "-" ] && lib=libkbengine.so
  ( export KB_ENGINE_LIB=$PWD/kafkabalancer_amd/lib/$lib
    IFS=','; for kv in $envs; do export "$kv"; done; unset IFS
    timeout -k 10 200 python3 -u bench.py --workload $WL --steps $STEPS --warmup 20 --no-cpu-baseline --no-secondary > $O/$name.out 2>&1 ) || { echo "$name failed"; tail -5 $O/$name.out; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/$name.out') if l.startswith('{')][0]
print('$name', round(d['ms_per_step']*1e3,2), {k: round(x,2) for k,x in d['kernels_us_per_launch'].items()}, d['engine_events'])"
done
