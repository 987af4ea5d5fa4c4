#!/bin/bash
# c2 / c3 step-body session: plain bench lines at the headline step counts plus the
# KB_STAMPS phase breakdown.  Usage: gpurun -- 'bash tools/gpu_c2.sh <tag>'
set -u
T=${1:-x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py --workload c2 --steps 100 --no-cpu-baseline > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python bench.py --workload c2 --steps 100 --no-cpu-baseline --stamps > $O/c2_stamps.json 2> $O/c2_stamps.err &&
timeout -k 10 300 python bench.py --steps 1000 --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --stamps > $O/c3_stamps.json 2> $O/c3_stamps.err
