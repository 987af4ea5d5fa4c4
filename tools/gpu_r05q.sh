set -u
O=gpurun_out/r05q
mkdir -p $O
P="env KB_ENGINE_LIB=kafkabalancer_amd/lib/libkbengine_prev.so KB_ABI_ANY=1"
b() { timeout -k 10 300 "$@" --no-cpu-baseline; }
b python bench.py --steps 1000 > $O/c3_cur1.json 2> $O/e1 &&
b $P python bench.py --steps 1000 > $O/c3_prev1.json 2> $O/e2 &&
b python bench.py --workload c2 --steps 100 > $O/c2_cur.json 2> $O/e3 &&
b $P python bench.py --workload c2 --steps 100 > $O/c2_prev.json 2> $O/e4 &&
b python bench.py --steps 1000 > $O/c3_cur2.json 2> $O/e5 &&
b $P python bench.py --steps 1000 > $O/c3_prev2.json 2> $O/e6 &&
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_fused.json 2> $O/e7 &&
KB_FUSE_SUM=0 timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_nofuse.json 2> $O/e8 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_sh -o sh -- python bench.py --sharded --steps 200 --warmup 20 > $O/rp_sh.log 2>&1 &&
KB_FUSE_SUM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_shn -o shn -- python bench.py --sharded --steps 200 --warmup 20 > $O/rp_shn.log 2>&1
