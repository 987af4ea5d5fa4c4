#!/bin/bash
# One GPU session: parity tests, then (only if the tests ended normally) the bench.
# Usage: tools/gpu_round.sh [tag] [pytest-args...]
TAG=${1:-r}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 600 "$@" > gpurun_out/gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_$TAG.log
case $rc in 0|1) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_$TAG.log
exit $rc
