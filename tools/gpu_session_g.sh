cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steps.py tests/test_golden_scale.py tests/test_gpu_incremental.py tests/test_gpu_fullsize.py -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r04g/pytest.log 2>&1; rc=$?
tail -8 gpurun_out/r04g/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/ablate.sh 64
