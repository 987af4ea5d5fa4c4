#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# bench lines of a measurement session into gpurun_out/$TAG/: the default bench (c3, with
# the CPU baseline), c2 / c4 / c5 / c3 at 1000 steps / c3nl / w16k (each with its CPU
# baseline), the drop-in costs at c3 and the
# rocprofv3 kernel-trace summaries of c3 and c2.  LINES overrides the list.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-lines}; mkdir -p $O
run() {   # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py "$@" > $O/$n.out 2>&1 || { echo "$n failed"; tail -5 $O/$n.out; exit 1; }
  grep -h '^{' $O/$n.out | tail -1 > $O/$n.json
  python3 -c "
import json; d=json.load(open('$O/$n.json'))
print('$n', {k: d.get(k) for k in ('value','ms_per_step','balance_per_call_us','steps_table_per_balance_us','plan_per_step_us')}, d.get('kernels_us_per_launch', ''), d.get('cli', ''))"
}
for l in ${LINES:-default c2 c4 c5 dropin prof}; do
  case $l in
    default) run default 400 ;;
    c2) run c2 300 --workload c2 --steps 80 --cpu-seconds 10 ;;
    c4) run c4 400 --workload c4 --steps 1000 --cpu-seconds 10 ;;
    c5) run c5 600 --workload c5 --steps 200 --cpu-seconds 10 ;;
    c3full) run c3full 400 --steps 1000 --cpu-seconds 10 ;;
    c3nl) run c3nl 400 --workload c3nl --steps 1000 --cpu-seconds 10 ;;
    w16k) run w16k 400 --workload w16k --steps 200 --cpu-seconds 10 ;;
    dropin) run dropin 500 --workload c3 --drop-in --steps 200 ;;
    prof) WLS="c3 c5" tools/prof_wl.sh > $O/prof.txt 2>&1 || { cat $O/prof.txt; exit 1; }
          cat $O/prof.txt
          for w in c3 c5; do cp $(find gpurun_out/prof/$w -name 'run_kernel_stats.csv' | head -1) $O/${w}_kernel_stats.csv
                             grep -h '^{' gpurun_out/prof/$w/bench.out | tail -1 > $O/${w}_bench_under_rocprof.json; done ;;
  esac
done
