cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u -m pytest tests/test_gpu_steps.py tests/test_shim_c.py tests/test_golden_scale.py -q -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r04d/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --stamps --steps 200 --warmup 20 > gpurun_out/r04d/stamps_c3.json 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c5 --steps 200 --warmup 10 --cpu-seconds 10 > gpurun_out/r04d/bench_c5.json 2> gpurun_out/r04d/bench_c5.err || exit $?
tail -c 1500 gpurun_out/r04d/stamps_c3.json
