#!/bin/bash
# round-3 measurement session: GPU parity suite, A/B against the previous build, then
# k_step alone on a fixed input for the production build and every -DKB_STOP_AT=k build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s3; mkdir -p $O
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
tools/exp_step.sh new=- prev=libkbengine_prev.so new2=- prev2=libkbengine_prev.so || exit 1
for w in ${WLS:-c3 c2}; do
  for lib in libkbengine.so $(for k in 1 2 3 4 5 6 7 8 9 10 11; do echo libkbengine_stop$k.so; done); do
    KB_STEP_LIB=$PWD/kafkabalancer_amd/lib/$lib timeout -k 10 120 python3 -u bench.py --workload $w --step-alone --steps 200 --warmup 20 > $O/alone_${w}_$lib.out 2>&1 || { tail -5 $O/alone_${w}_$lib.out; exit 1; }
    grep -h "^{" $O/alone_${w}_$lib.out
  done
done
