#!/bin/bash
# Round-4 closing measurements on the fused-pair tree: the whole -m gpu suite, then the bench
# lines of every config with CPU baselines and the rocprofv3 summaries of c3 / c5
# (tools/gpu_lines.sh).  Every GPU step has its own time limit; the chain stops at the first
# abnormal exit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; tail -4 $O/pytest_gpu_full.log
case $rc in 0|1) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
TAG=${TAG:-r04d} tools/gpu_lines.sh
