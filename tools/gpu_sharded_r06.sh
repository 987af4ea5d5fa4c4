#!/bin/bash
# The sharded protocol at world size 1 (bench.py --sharded: c3 and c5 against the plain
# plan), then the sharded / distributed GPU tests.  Usage: gpurun -- 'bash tools/gpu_sharded_r06.sh <tag>'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sh}; mkdir -p $O
timeout -k 10 200 python3 -u bench.py --sharded --workload c5 --steps 200 --warmup 20 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 200 python3 -u bench.py --sharded --workload c3 --steps 200 --warmup 20 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 600 python3 -u -m pytest tests/test_dist.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
cat $O/c5.json $O/c3.json; tail -3 $O/pytest.log
exit $rc
