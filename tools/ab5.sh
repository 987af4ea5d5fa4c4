#!/bin/bash
# A/B timing on one box for c3 and c5: tools/ab5.sh TAG libA.so libB.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=$1; A=$2; B=$3
for w in c3 c5; do
  st=1000; [ $w = c5 ] && st=200
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    KB_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --steps $st --warmup 5 --no-cpu-baseline > gpurun_out/ab_tmp.log 2>&1 || { tail -5 gpurun_out/ab_tmp.log; exit 1; }
    echo "$w $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_tmp.log) $(grep -o '"kernels_us_per_step": {[^}]*}' gpurun_out/ab_tmp.log)" >> gpurun_out/ab_$TAG.log
  done
done
exit 0
