#!/bin/bash
# Diagnostic: k_step time with phases run twice (kafkabalancer_amd/csrc `make rep REP=n`
# builds; results are unchanged, the extra time is the repeated phase's cost).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rep; mkdir -p $O
for v in "" $@; do
  lib=kafkabalancer_amd/lib/libkbengine${v:+_rep$v}.so
  KB_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/rep$v.out 2>&1 || { tail -5 $O/rep$v.out; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/rep$v.out') if l.startswith('{')][0]
print('rep=$v', round(d['ms_per_step']*1e3,2), {k: round(x,2) for k,x in d['kernels_us_per_step'].items()}, d['engine_events'])"
done
