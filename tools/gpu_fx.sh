#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# the whole -m gpu suite on the default (fused) path, then the exact-fold tests on the
# two-launch path (KB_FUSE=0); each step under its own time limit
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-fx}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; tail -6 $O/pytest_gpu_full.log
case $rc in 0|1) ;; *) echo "stopping: pytest rc=$rc"; exit $rc;; esac
KB_FUSE=0 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_exact_folds.py tests/test_gpu_fullsize.py > $O/pytest_nofuse.log 2>&1
echo "KB_FUSE=0: $(tail -1 $O/pytest_nofuse.log)"
