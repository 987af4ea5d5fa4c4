cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_dist; mkdir -p $O
KB_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --workload c3 --steps 100 --warmup 10 \
    --no-cpu-baseline > $O/gpus2_gloo_c3.out 2>&1 || { tail -5 $O/gpus2_gloo_c3.out; exit 1; }
grep -h '^{' $O/gpus2_gloo_c3.out | tail -1 > $O/gpus2_gloo_c3.json; head -c 400 $O/gpus2_gloo_c3.json
