#!/bin/bash
# The multi-GPU bench path on one GPU: bench.py --dist-world1 under a one-rank
# torch.distributed.run launch (RCCL) at full c3 and c5, and the two-rank gloo rehearsal
# (bench.py --gpus 2, both ranks on the box's one GPU, host-staged summaries) at full c3.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dist}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for wl in c3 c5; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $((29611 + RANDOM % 1000)) bench.py --dist-world1 --workload $wl --steps 200 --warmup 20 \
      --no-cpu-baseline > $O/dist_world1_$wl.out 2>&1 || { tail -5 $O/dist_world1_$wl.out; exit 1; }
  grep -h '^{' $O/dist_world1_$wl.out | tail -1 > $O/dist_world1_$wl.json
done
KB_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --workload c3 --steps 100 --warmup 10 \
    --no-cpu-baseline > $O/gpus2_gloo_c3.out 2>&1 || { tail -5 $O/gpus2_gloo_c3.out; exit 1; }
grep -h '^{' $O/gpus2_gloo_c3.out | tail -1 > $O/gpus2_gloo_c3.json
for f in $O/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', {k: d.get(k) for k in ('n_gpus','ms_per_step','value','scaling','exchange')}, d.get('roofline',{}).get('frac'))"; done
