#!/bin/bash
# Round-6 closing measurements into gpurun_out/$TAG: bench lines with CPU baselines (default c3
# with the c3nl secondary, c3 at 1000 steps, c2, c3nl at 1000 steps, c5), the drop-in costs,
# rocprofv3 kernel-trace summaries of c3 and c5 (tools/gpu_lines.sh), then the smoke test.
# Usage: gpurun -- 'TAG=r06_m2 bash tools/gpu_r06_close.sh'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export TAG=${TAG:-r06_close}
LINES=${LINES:-"default c3full c2 c3nl c5 dropin prof"} bash tools/gpu_lines.sh || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
