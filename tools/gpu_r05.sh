#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Round-5 GPU session (run through gpurun from the repo root): the bench lines of the
# headline and the c2 / c3nl / c5 / sharded workloads, then the GPU suite.
# Usage: gpurun -- 'bash tools/gpu_r05.sh <tag> [steps]'
set -u
T=${1:-x}
S=${2:-200}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py --workload c2 --steps $S --no-cpu-baseline > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python bench.py --workload c3nl --steps $S --no-cpu-baseline > $O/c3nl.json 2> $O/c3nl.err &&
timeout -k 10 300 python bench.py --steps $S --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python bench.py --workload c5 --steps $S --no-cpu-baseline > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python bench.py --sharded --steps $S --warmup 20 > $O/sharded.json 2> $O/sharded.err &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
