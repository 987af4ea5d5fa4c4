#!/bin/bash
# A/B of the production build against lib/libkbengine_base.so on c3 / c3nl (alternated), then
# a parity subset ($TESTS).  Usage: gpurun -- 'bash tools/session_ab.sh TAG'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-ab}; O=gpurun_out/$T; mkdir -p $O
export KB_DIAGNOSTICS=1 KB_ABI_ANY=1
for wl in ${WLS:-c3 c3nl}; do
  WL=$wl STEPS=${STEPS:-1000} timeout -k 10 500 bash tools/exp_step.sh ${SPECS:-base=libkbengine_base.so new=- base2=libkbengine_base.so new2=-} > $O/ab_$wl.txt 2>&1 || { cat $O/ab_$wl.txt; exit 1; }
  echo "== $wl"; cat $O/ab_$wl.txt
done
[ "${TESTS:-}" = none ] && exit 0
timeout -k 10 800 python3 -u -m pytest ${TESTS:-tests/test_golden_scale.py tests/test_gpu_fused.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; exit $rc
