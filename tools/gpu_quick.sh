#!/bin/bash
# Quick GPU session: -m gpu tests, one c3 bench line, optional extra bench args / stamps run.
# Usage: tools/gpu_quick.sh TAG [--notest] [--stamps] [--c5]
TAG=${1:-q}; shift
TEST=1; STAMPS=0; C5=0
for a in "$@"; do
  case $a in --notest) TEST=0;; --stamps) STAMPS=1;; --c5) C5=1;; esac
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
run() { local name=$1 lim=$2; shift 2; echo "== $name: $*" >> $O/log.txt; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ] || { tail -30 $O/$name.out; exit $rc; }; }
[ $TEST -eq 1 ] && run tests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run c3 300 python3 -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline
[ $STAMPS -eq 1 ] && run stamps_c3 300 python3 -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --stamps
[ $C5 -eq 1 ] && run c5 400 python3 -u bench.py --workload c5 --steps 200 --warmup 5 --no-cpu-baseline
[ $C5 -eq 1 ] && [ $STAMPS -eq 1 ] && run stamps_c5 400 python3 -u bench.py --workload c5 --steps 200 --warmup 5 --no-cpu-baseline --stamps
tail -3 $O/tests.out 2>/dev/null; grep -h '^{' $O/*.out | cut -c1-400
echo ALLDONE
