#!/bin/bash
# Diagnostic: instruction-cache counters of the c3 bench's kernels (one rocprofv3 pass).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-icache}
timeout -k 5 -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_avail.txt 2>&1
grep -o 'SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_VALU\b\|SQ_WAIT_INST_ANY\|SQ_INST_CYCLES[A-Z_]*' gpurun_out/${TAG}_avail.txt | sort -u > gpurun_out/${TAG}_names.txt
cat gpurun_out/${TAG}_names.txt
timeout -k 5 -s KILL 150 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/${TAG}_ic -o run \
    -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/${TAG}_ic.log 2>&1 || exit $?
exit 0
