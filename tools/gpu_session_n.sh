#!/bin/bash
# Closing measurements of round 4 on the final tree: the eager-workgroup phase diagnostic
# (a -DKB instrumented variant, tools/eager_diag.py), the bench lines of every config with
# CPU baselines and the rocprofv3 summaries (tools/gpu_lines.sh), then the PMC passes for
# the roofline's traffic (tools/pmc_r04.sh).  Each step under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04n}; mkdir -p $O
if [ -f kafkabalancer_amd/lib/libkbengine_diag2.so ]; then
  KB_ENGINE_LIB=$PWD/kafkabalancer_amd/lib/libkbengine_diag2.so timeout -k 10 240 python3 -u tools/eager_diag.py c5 100 > $O/eager_diag.json 2> $O/eager_diag.err || { echo "diag failed"; tail -3 $O/eager_diag.err; exit 1; }
  cat $O/eager_diag.json
fi
TAG=${TAG:-r04n} tools/gpu_lines.sh || exit 1
[ -n "$HEAD" ] && { tools/pmc_r04.sh $HEAD c3 c5 || exit 1; }
exit 0
