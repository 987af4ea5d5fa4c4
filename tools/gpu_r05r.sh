set -u
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_fd.log 2>&1 &&
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_fused.json 2> $O/e7 &&
KB_FUSE_SUM=0 timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_nofuse.json 2> $O/e8 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_sh -o sh -- python bench.py --sharded --steps 200 --warmup 20 > $O/rp_sh.log 2>&1
