#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Quick check of a build on one box: bench lines (200 steps, no CPU baseline) of the
# workloads in $WLS, then the GPU tests in $TESTS (default: the fused-pair, full-size pin,
# parity and per-step files; TESTS=all runs the whole -m gpu suite).
# Usage: gpurun -- 'bash tools/gpu_quick.sh <tag>'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T; mkdir -p $O
WLS=${WLS:-c3 c3nl c5 c4 c2}
TESTS=${TESTS:-tests/test_gpu_fused.py tests/test_golden_scale.py tests/test_gpu_parity.py tests/test_gpu_steps.py}
[ "$TESTS" = all ] && TESTS=tests
for wl in $WLS; do
  timeout -k 10 200 python3 -u bench.py --workload $wl --steps 200 --warmup 20 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
done
python3 tools/show_r05.py $O
[ "$TESTS" = none ] && exit 0
timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
