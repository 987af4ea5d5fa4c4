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
world = int(os.environ.get("PROBE_WORLD", "2"))
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
plan = [[], []]
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
        if os.environ.get("PROBE_DUMP") and step == 0:
            import numpy as np
            g = gathered.cpu().numpy()
            for r in range(world):
                h = g[r * nb:r * nb + 112]
                d = np.frombuffer(h[:16].tobytes(), np.float64)
                c = np.frombuffer(h[16:32].tobytes(), np.uint64)
                u = np.frombuffer(h[32:44].tobytes(), np.uint32)
                k = np.frombuffer(h[44:48].tobytes(), np.uint16)
                print("rank", r, "dmin", d, "cand", c, "nkeys/flags/fmask", u, "nkk", k, flush=True)
                for kk in range(2):
                    b = h[48 + 32 * kk:80 + 32 * kk].tobytes()
                    st = np.frombuffer(b[:8], np.int32); w = np.frombuffer(b[8:16], np.float64)
                    it = np.frombuffer(b[16:24], np.uint64); kd = np.frombuffer(b[24:28], np.int32)
                    print("   best", kk, "s,t", st, "w", w, "part", int(it[0]) >> 21, "slot", (int(it[0]) >> 16) & 31, "kind", kd, flush=True)
                ko = r * nb + 112 + 32
                for q in range(int(u[0])):
                    b = g[ko + 32 * q: ko + 32 * q + 32].tobytes()
                    st = np.frombuffer(b[:8], np.int32); it = np.frombuffer(b[16:24], np.uint64); kd = np.frombuffer(b[24:28], np.int32)
                    print("   key", q, "s,t", st, "part", int(it[0]) >> 21, "slot", (int(it[0]) >> 16) & 31, "kind", kd, flush=True)
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
    for r in range(world):
        plan[r].extend(res[r][1])
    if all(s == "done" for s, _ in res):
        break
    chk("collect")
from helpers import oracle_plan, key
och, oerr, opl = oracle_plan(synth.to_plist(cl), cfg, len(plan[0]))
a = [key(c) for c in plan[0]]
b = [key(c) for c in och]
print("ranks agree:", [key(c) for c in plan[1]] == a, "plan == oracle:", a == b, len(a), len(b), flush=True)
for i, (x, y) in enumerate(zip(a, b)):
    if x != y:
        print("first diff", i, x, y, flush=True)
        break
print("OK", flush=True)
