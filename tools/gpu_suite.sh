#!/bin/bash
# The whole GPU test suite into gpurun_out/$1/pytest_gpu.log.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; exit $rc
