#!/bin/bash
# A/B timing on one box: tools/ab.sh TAG libA.so libB.so [rounds]
# Runs the c3 bench alternately with each engine library (KB_ENGINE_LIB); AB_ENV_A /
# AB_ENV_B add one VAR=value to the environment of the A / B runs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=$1; A=$2; B=$3; R=${4:-2}
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; envv=${AB_ENV_A:-X=0}; [ $v = B ] && { lib=$B; envv=${AB_ENV_B:-X=0}; }
    env $envv KB_ENGINE_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/ab_tmp.log 2>&1 || { tail -5 gpurun_out/ab_tmp.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_tmp.log) $(grep -o '"kernels_us_per_step": {[^}]*}' gpurun_out/ab_tmp.log)" >> gpurun_out/ab_$TAG.log
  done
done
exit 0
