#!/bin/bash
# the whole -m gpu suite, then the default and c5 bench lines (tools/gpu_lines.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; tail -4 $O/pytest_gpu_full.log
case $rc in 0|1) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
TAG=${TAG:-r04m} LINES=${LINES:-"default c5"} tools/gpu_lines.sh
