#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# A/B of the fused pair (k_pair) against the two-launch pair on the default bench, then the
# parity tests that run plans through it.  Every GPU step has its own time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-fuse}; mkdir -p $O
for f in 1 0; do
  KB_FUSE=$f timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench_fuse$f.json 2> $O/bench_fuse$f.err || { echo "bench fuse=$f failed"; tail -5 $O/bench_fuse$f.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_fuse$f.json').read().strip().splitlines()[-1])
print('fuse=$f', d['ms_per_step'], d.get('kernels_us_per_launch'), d.get('engine_events'), d['config'].get('fused_pairs'))"
done
[ -n "$NOTEST" ] && exit 0
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread ${TESTS:-tests/test_golden_scale.py tests/test_gpu_parity.py tests/test_gpu_steps.py} > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; exit $rc
