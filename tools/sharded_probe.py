"""Diagnostic: the two-shard batched protocol of tests/test_dist.py with a device-wide
synchronisation after every engine call, printing the first call that fails."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from kafkabalancer_amd import engine as E
from kafkabalancer_amd import synth
from kafkabalancer_amd.dist import shard_bounds
from helpers import default_cfg

cl = synth.make_cluster(2500, 40, 3, "zipf", nsets=8, set_size=24, seed=5, with_names=True)
cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
world = 2
engs = [E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, r)) for r in range(world)]
print("shards", [shard_bounds(cl.n, world, r) for r in range(world)], "stats", [e.stats()["scan_workgroups"] for e in engs], flush=True)
nb = engs[0].summary_bytes()
summ = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
gathered = torch.zeros(world * nb, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()


SYNC = os.environ.get("PROBE_SYNC", "1") == "1"


def chk(what):
    if not SYNC and what != "collect":
        return
    try:
        torch.cuda.synchronize()
    except Exception as ex:
        print("FAILED after", what, repr(ex)[:120], flush=True)
        sys.exit(3)


step = 0
for batch_no in range(4):
    for r, e in enumerate(engs):
        print("reset r%d" % r, flush=True)
        e.sharded_reset(8)
        chk("reset r%d" % r)
    for _ in range(8):
        for r, (e, b) in enumerate(zip(engs, summ)):
            e.sharded_scan(b.data_ptr())
            chk("scan r%d step %d" % (r, step))
        torch.cuda.synchronize()                  # (as the test: the scans, then the copies)
        for r in range(world):
            gathered[r * nb:(r + 1) * nb].copy_(summ[r])
        torch.cuda.synchronize()
        chk("gather step %d" % step)
        for r, e in enumerate(engs):
            print("resolve r%d step %d" % (r, step), flush=True)
            e.sharded_resolve(gathered.data_ptr(), world)
            chk("resolve r%d step %d" % (r, step))
        step += 1
    res = []
    for r, e in enumerate(engs):
        print("collect r%d" % r, flush=True)
        res.append(e.sharded_collect(9))
    print("batch", batch_no, [(s, len(c)) for s, c in res], flush=True)
    chk("collect")
print("OK", flush=True)
