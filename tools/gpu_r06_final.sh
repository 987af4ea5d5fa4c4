#!/bin/bash
# Round-6 final measurements into gpurun_out/$TAG: the bench lines (tools/gpu_lines.sh: default
# c3 with the c3nl secondary, c3 at 1000 steps, c2, c3nl, c4, c5, the drop-in costs, rocprofv3
# kernel-trace summaries of c3 and c5), the world-1 sharded lines of c3 and c5, then smoke().
# Usage: gpurun -- 'TAG=r06_final bash tools/gpu_r06_final.sh'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export TAG=${TAG:-r06_final}
O=gpurun_out/$TAG; mkdir -p $O
LINES=${LINES:-"default c3full c2 c3nl c4 c5 dropin prof"} bash tools/gpu_lines.sh || exit 1
for wl in c3 c5; do
  timeout -k 10 300 python3 -u bench.py --sharded --workload $wl --steps 200 --warmup 20 > $O/sharded_$wl.out 2>&1 || { tail -5 $O/sharded_$wl.out; exit 1; }
  grep -h '^{' $O/sharded_$wl.out | tail -1 > $O/sharded_$wl.json; cat $O/sharded_$wl.json
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
