#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Round-4 GPU session: the whole -m gpu suite (no -x: every failure is listed), then --
# only if it ended normally -- the default bench line and a rocprofv3 kernel trace of the
# same command.  Every GPU step has its own time limit; the chain stops at the first
# abnormal exit (fault, abort, timeout).
# Usage: tools/gpu_r04.sh TAG [--notest] [--nobench] [--prof] [pytest-args...]
TAG=${1:-r04}; shift
TEST=1; BENCH=1; PROF=0
while [ "${1#--}" != "$1" ] && [ "$1" = "--notest" -o "$1" = "--nobench" -o "$1" = "--prof" ]; do
  [ "$1" = "--notest" ] && TEST=0
  [ "$1" = "--nobench" ] && BENCH=0
  [ "$1" = "--prof" ] && PROF=1
  shift
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/$TAG
if [ $TEST -eq 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -q -v -m gpu --timeout 240 --timeout-method thread "$@" \
      > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/$TAG/pytest_gpu.log
  tail -25 gpurun_out/$TAG/pytest_gpu.log
  case $rc in 0|1|5) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
fi
if [ $BENCH -eq 1 ]; then
  timeout -k 10 400 python -u bench.py --cpu-seconds 10 > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err
  rc=$?
  echo "bench rc=$rc"; tail -c 3000 gpurun_out/$TAG/bench_default.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ $PROF -eq 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o c3 \
      -- python3 bench.py --no-cpu-baseline > gpurun_out/$TAG/prof_c3.json 2> gpurun_out/$TAG/prof_c3.err
  rc=$?
  echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
