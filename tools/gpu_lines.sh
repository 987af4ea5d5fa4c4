#!/bin/bash
# bench lines of a measurement session into gpurun_out/$TAG/: the default bench (c3, with
# the CPU baseline), c2 / c4 / c5 (no CPU baseline), the drop-in costs at c3 and the
# rocprofv3 kernel-trace summaries of c3 and c2.  LINES overrides the list.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-lines}; mkdir -p $O
run() {   # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py "$@" > $O/$n.out 2>&1 || { echo "$n failed"; tail -5 $O/$n.out; exit 1; }
  grep -h '^{' $O/$n.out | tail -1 > $O/$n.json
  python3 -c "
import json; d=json.load(open('$O/$n.json'))
print('$n', {k: d.get(k) for k in ('value','ms_per_step','balance_per_call_us','plan_per_step_us')}, d.get('kernels_us_per_step', ''), d.get('cli', ''))"
}
for l in ${LINES:-default c2 c4 c5 dropin prof}; do
  case $l in
    default) run default 400 ;;
    c2) run c2 200 --workload c2 --steps 80 --no-cpu-baseline ;;
    c4) run c4 300 --workload c4 --steps 1000 --no-cpu-baseline ;;
    c5) run c5 500 --workload c5 --steps 200 --no-cpu-baseline ;;
    dropin) run dropin 500 --workload c3 --drop-in --steps 200 ;;
    prof) WLS="c3 c2" tools/prof_wl.sh > $O/prof.txt 2>&1 || { cat $O/prof.txt; exit 1; }
          cat $O/prof.txt; cp gpurun_out/prof/c3/run_kernel_stats.csv $O/c3_kernel_stats.csv
          cp gpurun_out/prof/c2/run_kernel_stats.csv $O/c2_kernel_stats.csv ;;
  esac
done
