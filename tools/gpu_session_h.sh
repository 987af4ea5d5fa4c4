cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r04h/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
STEPS=600 WL=c3 bash tools/exp_step.sh base=libkbengine_base.so frz=libkbengine_frz.so head=- headnobk=-:KB_STEP_BK=0 abl64=libkbengine_abl64.so base2=libkbengine_base.so head2=- abl64b=libkbengine_abl64.so || exit 1
STEPS=200 WL=c5 bash tools/exp_step.sh base=libkbengine_base.so head=- lazy=-:KB_EAGER=0 || exit 1
