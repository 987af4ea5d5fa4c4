#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Round-6 GPU session: the driver's default bench line (c3 + the c3nl secondary, CPU legs),
# optional extra workloads ($WLS, 200 steps, no CPU leg), then the GPU suite ($TESTS: a file
# list, `all` (default) or `none`).
# Usage: gpurun -- 'bash tools/gpu_r06.sh <tag>'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r6}
O=gpurun_out/$T; mkdir -p $O
TESTS=${TESTS:-all}
[ "$TESTS" = all ] && TESTS=tests
timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $O/default.json 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
for wl in ${WLS:-}; do
  timeout -k 10 200 python3 -u bench.py --workload $wl --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
done
[ "$TESTS" = none ] && exit 0
timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
