#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Step-body session: bench lines of c2 / c3 / c3nl / c5 at their headline step counts, the
# sharded world-1 line with and without the fused summary, the KB_STAMPS phase breakdown of c2 and c3, then the GPU suite.
# Usage: gpurun -- 'bash tools/gpu_c2.sh <tag> [suite]'
set -u
T=${1:-x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py --workload c2 --steps 100 --no-cpu-baseline > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python bench.py --steps 1000 --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python bench.py --steps 1000 --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err &&
timeout -k 10 300 python bench.py --workload c3nl --steps 1000 --no-cpu-baseline > $O/c3nl.json 2> $O/c3nl.err &&
timeout -k 10 300 python bench.py --workload c5 --steps 200 --no-cpu-baseline > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sharded.json 2> $O/sharded.err &&
KB_FUSE_SUM=0 timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sharded_nofuse.json 2> $O/sharded_nofuse.err &&
timeout -k 10 300 python bench.py --workload c2 --steps 100 --no-cpu-baseline --stamps > $O/c2_stamps.json 2> $O/c2_stamps.err &&
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --stamps > $O/c3_stamps.json 2> $O/c3_stamps.err &&
if [ "${2:-}" = suite ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
fi
