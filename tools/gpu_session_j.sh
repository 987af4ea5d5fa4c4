cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=600 WL=c3 bash tools/exp_step.sh frz=libkbengine_frz.so head=- noeg=libkbengine_noeg.so frz2=libkbengine_frz.so head2=- noeg2=libkbengine_noeg.so || exit 1
