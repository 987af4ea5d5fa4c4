cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r04i/pytest.log 2>&1; rc=$?
tail -6 gpurun_out/r04i/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
STEPS=600 WL=c3 bash tools/exp_step.sh frz=libkbengine_frz.so head=- frz2=libkbengine_frz.so head2=- || exit 1
STEPS=200 WL=c5 bash tools/exp_step.sh base=libkbengine_base.so head=- lazy=-:KB_EAGER=0 head2=- || exit 1
