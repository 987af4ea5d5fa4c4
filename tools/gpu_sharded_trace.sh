#!/bin/bash
# Kernel trace of the world-1 sharded c3 line, then the sharded GPU tests of tests/test_dist.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sht}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 -u bench.py --sharded --workload c3 --steps 100 --warmup 10 > $O/c3_prof.json 2> $O/c3_prof.err &&
timeout -k 10 600 python3 -u -m pytest tests/test_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log; exit $rc
