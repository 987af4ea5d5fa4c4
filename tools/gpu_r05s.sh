set -u
O=gpurun_out/r05s
mkdir -p $O
b() { timeout -k 10 300 "$@" --no-cpu-baseline; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_fd.log 2>&1 &&
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_fused.json 2> $O/e7 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_sh -o sh -- python bench.py --sharded --steps 200 --warmup 20 > $O/rp_sh.log 2>&1 &&
b python bench.py --workload c3nl --steps 1000 > $O/c3nl_1000.json 2> $O/e1 &&
KB_EAGER=1 b python bench.py --workload c3nl --steps 1000 > $O/c3nl_1000_eager.json 2> $O/e2 &&
b python bench.py --workload c3nl --steps 200 > $O/c3nl_200.json 2> $O/e3 &&
KB_EAGER=1 b python bench.py --workload c3nl --steps 200 > $O/c3nl_200_eager.json 2> $O/e4 &&
KB_EAGER=1 b python bench.py --steps 1000 > $O/c3_eager.json 2> $O/e5
