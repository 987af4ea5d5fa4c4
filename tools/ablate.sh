#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Diagnostic: k_step time with phases ablated (kafkabalancer_amd/csrc `make abl ABL=n`
# builds; their plans are wrong by construction, only the timing is of interest).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/abl; mkdir -p $O
for v in "" $@; do
  lib=kafkabalancer_amd/lib/libkbengine${v:+_abl$v}.so
  KB_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/abl$v.out 2>&1 || { tail -5 $O/abl$v.out; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/abl$v.out') if l.startswith('{')][0]
print('abl=$v', round(d['ms_per_step']*1e3,2), {k: round(x,2) for k,x in d['kernels_us_per_launch'].items()}, d['engine_events'])"
done
