#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# One GPU session: parity tests, then (only if the tests ended normally) the
# bench, then (optionally) a rocprofv3 kernel-trace of the bench and PMC passes.
# Usage: tools/gpu_round.sh TAG [--prof] [--pmc] [--notest] [pytest-args...]
TAG=${1:-r}; shift
PROF=0; PMC=0; TEST=1
while [ "$1" = "--prof" ] || [ "$1" = "--pmc" ] || [ "$1" = "--notest" ]; do
  [ "$1" = "--prof" ] && PROF=1
  [ "$1" = "--pmc" ] && PMC=1
  [ "$1" = "--notest" ] && TEST=0
  shift
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
if [ $TEST -eq 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread "$@" \
      > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/gpu_$TAG.log
  case $rc in 0|1|5) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
  [ $rc -eq 1 ] && { echo "tests failed"; tail -30 gpurun_out/gpu_$TAG.log; exit 1; }
fi
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --cpu-seconds 10 > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ $PROF -eq 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
      -- python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  rc=$?
  echo "rocprof rc=$rc" >> gpurun_out/prof_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ $PMC -eq 1 ]; then
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$TAG -o fetch \
      -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/pmc_$TAG.log 2>&1 || exit $?
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_$TAG -o write \
      -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline >> gpurun_out/pmc_$TAG.log 2>&1 || exit $?
fi
exit 0
