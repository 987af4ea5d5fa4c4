#!/bin/bash
# Diagnostic: rocprofv3 PC sampling of the c3 bench (where k_step's waves spend time).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pcs; mkdir -p $O
M=${1:-host_trap}; U=${2:-time}; I=${3:-1}
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
    --pc-sampling-interval $I --kernel-trace --output-format csv -d $O/$M -o run \
    -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > $O/$M.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 $O/$M.log; ls -la $O/$M; exit $rc
