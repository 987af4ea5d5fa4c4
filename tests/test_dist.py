"""Multi-rank plan protocol (kafkabalancer_amd/dist.py).

CPU: world_size-2 gloo run of ShardedPlanner with a CPU engine that follows the
same summary protocol (each rank scores its shard exactly, the merge takes the
lexicographic (U, iteration) minimum) -- checks the exchange and that every
rank applies the identical change, against the single-process oracle plan.

GPU: two device engines on disjoint shards of one cluster on one GPU, their
summaries concatenated as the all-gather would, against one unsharded engine.
"""
import json
import os
import random
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kafkabalancer_amd.dist import ShardedPlanner, shard_bounds
from oracle import pyref

from helpers import default_cfg


def _cluster(seed, P=40, B=6):
    rng = random.Random(seed)
    parts = []
    for i in range(P):
        reps = rng.sample(range(1, B + 1), 3)
        parts.append({"topic": "t", "partition": i, "replicas": reps,
                      "weight": float(rng.randint(1, 4))})
    return {"version": 1, "partitions": parts}


class CpuShardEngine:
    """Exact move() restricted to a shard (steps.go:210-297), summary = (U, iter)."""

    def __init__(self, plist, cfg, begin, end):
        self.pl = pyref.normalize(plist)
        pyref.balance([dict(p, replicas=list(p["replicas"])) for p in self.pl], cfg)  # validates
        self.cfg = cfg
        self.begin, self.end = begin, end
        # FillDefaults on the local state
        for p in self.pl:
            p["brokers"] = sorted({r for q in self.pl for r in q["replicas"]}) if p["brokers"] is None else p["brokers"]
            p["num_replicas"] = p["num_replicas"] or len(p["replicas"])

    def summary_bytes(self):
        return 4 * 8

    def step_begin(self, summary):
        loads = pyref.broker_load(self.pl)
        bl = pyref.get_bl(loads)
        su = pyref.unbalance(bl)
        best = (float("inf"), float("inf"), -1.0, -1.0)
        for i in range(self.begin, self.end):
            p = self.pl[i]
            if p["num_replicas"] < self.cfg["min_replicas"]:
                continue
            for slot in range(1, len(p["replicas"])):
                r = p["replicas"][slot]
                ridx = [k for k, x in enumerate(bl) if x[0] == r][0]
                rl = bl[ridx][1]
                bl[ridx][1] -= p["weight"]
                for k, (b, l) in enumerate(bl):
                    if b not in p["brokers"] or b in p["replicas"]:
                        continue
                    bl[k][1] = l + p["weight"]
                    u = pyref.unbalance(bl)
                    it = (i * 32 + slot) * 4096 + k
                    if (u, it) < best[:2]:
                        best = (u, float(it), float(i), float(b))
                    bl[k][1] = l
                bl[ridx][1] = rl
        self.su = su
        summary.copy_(torch.from_numpy(np.array(best, np.float64)).view(torch.uint8))

    def step_finish(self, gathered, world):
        recs = gathered.view(torch.float64).reshape(world, 4).tolist()
        u, it, i, b = min(recs, key=lambda x: (x[0], x[1]))
        if not (u < self.su - self.cfg["min_unbalance"]):
            return None
        i, b = int(i), int(b)
        slot = (int(it) // 4096) % 32
        p = self.pl[i]
        frm = p["replicas"][slot]
        p["replicas"][slot] = b
        return {"pidx": i, "slot": slot, "from_": frm, "to": b}


def _worker(rank, world, port, plist, cfg, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = len(plist["partitions"])
    # shard on small tiles for the test (the device engine uses 1024)
    per = -(-n // world)
    begin, end = rank * per, min(n, (rank + 1) * per)
    eng = CpuShardEngine(plist, cfg, begin, end)
    sp = ShardedPlanner(eng, world, device_tensors=False)
    out = sp.plan(steps)
    q.put((rank, [(c["pidx"], c["slot"], c["from_"], c["to"]) for c in out],
           [p["replicas"] for p in eng.pl]))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("seed", [1, 2])
def test_gloo_two_ranks_match_single_process(seed):
    plist = _cluster(seed)
    cfg = default_cfg(min_unbalance=0.0)
    steps = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, plist, cfg, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (ch, st)) for r, ch, st in [q.get(timeout=300) for _ in procs])
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1]                      # every rank applied the identical plan
    # the single-process reference plan
    pl = pyref.normalize(plist)
    want = []
    for _ in range(steps):
        r = pyref.balance(pl, cfg)
        if r is None:
            break
        want.append((r[1], r[3], r[4]))
    got = [(i, f, t) for i, _, f, t in res[0][0]]
    assert got == want
    assert res[0][1] == [p["replicas"] for p in pl]


def test_shard_bounds_cover_and_align():
    for n in [1, 1000, 1024, 5000, 1_000_001]:
        for world in [1, 2, 3, 8]:
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            assert all(a % 1024 == 0 or a == b for a, b in spans)   # aligned or empty


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["zipf-sets", "uniform"])
def test_two_engines_one_gpu_match_unsharded(workload):
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    if workload == "zipf-sets":
        cl = synth.make_cluster(5000, 200, 3, "zipf", nsets=16, set_size=40, seed=3)
        cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
    else:
        cl = synth.make_cluster(5000, 60, 3, "uniform", seed=4)
        cfg = default_cfg(min_unbalance=0.0)
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(30)
    assert err is None
    world = 2
    engs = [E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, r)) for r in range(world)]
    got, grows = [], 0
    bufs = None
    while len(got) < 30:
        nb = engs[0].summary_bytes()                 # (grows when a summary overflows)
        if bufs is None or bufs[0].numel() != nb:
            bufs = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
            torch.cuda.synchronize()
        for e, b in zip(engs, bufs):
            e.step_begin(b.data_ptr())
        torch.cuda.synchronize()
        gathered = torch.cat(bufs)
        chs = [e.step_finish(gathered.data_ptr(), world) for e in engs]
        assert chs[0] == chs[1]
        if chs[0] in ("retry", "grow"):               # the same step again
            grows += chs[0] == "grow"
            continue
        if chs[0] is None:
            break
        got.append(chs[0])
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert [key(c) for c in got] == [key(c) for c in want]
    assert engs[0].state() == ref.state() == engs[1].state()



@pytest.mark.gpu
def test_two_engines_one_gpu_batched_protocol():
    """The batched sharded protocol (sharded_reset / scan / resolve / collect: no host
    round trip per step) gives the unsharded plan."""
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    cl = synth.make_cluster(5000, 200, 3, "zipf", nsets=16, set_size=40, seed=3)
    cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(40)
    assert err is None
    world = 2
    engs = [E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, r)) for r in range(world)]
    got = [[], []]
    done = False
    while not done and len(got[0]) < 40:
        nb = engs[0].summary_bytes()
        batch = min(16, 40 - len(got[0]))
        for e in engs:
            e.sharded_reset(batch)
        # every buffer of the batch exists (and is zeroed) before the engines' streams
        # write into them
        allb = [[torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)] for _ in range(batch)]
        torch.cuda.synchronize()
        keep = []
        for bufs in allb:
            for e, b in zip(engs, bufs):
                e.sharded_scan(b.data_ptr())
            torch.cuda.synchronize()
            gathered = torch.cat(bufs)
            torch.cuda.synchronize()                   # the engines' streams read it next
            keep.append((bufs, gathered))
            for e in engs:
                e.sharded_resolve(gathered.data_ptr(), world)
        res = [e.sharded_collect(batch + 1) for e in engs]
        assert res[0][0] == res[1][0]
        for r in range(world):
            got[r].extend(res[r][1])
        done = res[0][0] == "done"
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert [key(c) for c in got[0]] == [key(c) for c in got[1]]
    assert [key(c) for c in got[0]][:40] == [key(c) for c in want][:len(got[0][:40])]
    assert len(got[0]) == len(want)
    assert engs[0].state() == ref.state() == engs[1].state()




def _protocol_plan(cl, cfg, world, steps):
    """The batched protocol with host-staged summaries over `world` shards of one process:
    (the plan of rank 0, every rank's plan, every engine's final state)."""
    from kafkabalancer_amd import engine as E
    engs = [E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, r)) for r in range(world)]
    got = [[] for _ in range(world)]
    done = False
    while not done and len(got[0]) < steps:
        nb = engs[0].summary_bytes()
        summ = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
        gathered = torch.zeros(world * nb, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        batch = min(8, steps - len(got[0]))
        for e in engs:
            e.sharded_reset(batch)
        for _ in range(batch):
            for e, b in zip(engs, summ):
                e.sharded_scan(b.data_ptr())
            torch.cuda.synchronize()
            for r in range(world):
                gathered[r * nb:(r + 1) * nb].copy_(summ[r])
            torch.cuda.synchronize()
            for e in engs:
                e.sharded_resolve(gathered.data_ptr(), world)
            torch.cuda.synchronize()
        res = [e.sharded_collect(batch + 1) for e in engs]
        assert len({st for st, _ in res}) == 1, [st for st, _ in res]
        for r in range(world):
            got[r].extend(res[r][1])
        done = res[0][0] == "done"
    states = [e.state() for e in engs]
    grows = [e.stats()["spill_grows"] for e in engs]
    for e in engs:
        e.close()
    return got, states, grows


@pytest.mark.gpu
def test_sharded_protocol_wide_brokers_two_shards_matches_plain():
    """Two shards at 2500 brokers: each rank's tightening bound pass sets its own census
    bound from its own shard (the ranks' bounds differ), yet both ranks apply the same plan
    -- the plain engine's -- and end in its state, with no spill growth."""
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    cl = synth.make_cluster(20000, 2500, 3, "zipf", seed=0x5EED00B6)
    cfg = default_cfg(allow_leader=False, min_unbalance=0.0)
    steps = 24
    got, states, grows = _protocol_plan(cl, cfg, 2, steps)
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(steps)
    assert err is None, err
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert [key(c) for c in got[1]] == [key(c) for c in got[0]]
    assert [key(c) for c in got[0]] == [key(c) for c in want]
    assert states[0] == states[1] == ref.state()
    assert grows == [0, 0]
    ref.close()


def _gpu_cluster():
    from kafkabalancer_amd import synth
    cl = synth.make_cluster(2500, 40, 3, "zipf", nsets=8, set_size=24, seed=5, with_names=True)
    return cl, default_cfg(allow_leader=True, min_unbalance=0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_sharded_protocol_matches_oracle(world):
    """One or two shards ([0, 2048) and the 452-partition tail) driven through the
    batched protocol with host-staged summaries (the gloo rehearsal's exchange), against
    the oracle's plan (oracle/kb_oracle.c), not the unsharded engine.  (Pins the fix of
    round 2: rank summaries take the key path -- a summary's best key need not be its
    one near-tie key when the first step's census spilled.)"""
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    from helpers import oracle_plan
    cl, cfg = _gpu_cluster()
    steps = 24
    engs = [E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, r)) for r in range(world)]
    got = [[] for _ in range(world)]
    done = False
    while not done and len(got[0]) < steps:
        nb = engs[0].summary_bytes()                 # (grows when a summary overflows)
        summ = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
        gathered = torch.zeros(world * nb, dtype=torch.uint8, device="cuda")
        h_gathered = torch.zeros(world * nb, dtype=torch.uint8)
        torch.cuda.synchronize()
        batch = min(8, steps - len(got[0]))
        for e in engs:
            e.sharded_reset(batch)
        for _ in range(batch):
            for e, b in zip(engs, summ):
                e.sharded_scan(b.data_ptr())
            torch.cuda.synchronize()
            for r in range(world):                     # staged: device -> host -> device
                h_gathered[r * nb:(r + 1) * nb].copy_(summ[r])
            gathered.copy_(h_gathered)
            torch.cuda.synchronize()
            for e in engs:
                e.sharded_resolve(gathered.data_ptr(), world)
            torch.cuda.synchronize()
        res = [e.sharded_collect(batch + 1) for e in engs]
        assert len({st for st, _ in res}) == 1, [st for st, _ in res]
        for r in range(world):
            got[r].extend(res[r][1])
        done = res[0][0] == "done"
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    for r in range(1, world):
        assert [key(c) for c in got[r]] == [key(c) for c in got[0]]
    pl = synth.to_plist(cl)
    och, oerr, opl = oracle_plan(pl, cfg, steps)
    assert oerr is None
    assert [key(c) for c in got[0]][:steps] == [key(c) for c in och]
    for e in engs:
        assert e.state() == opl.state()


def _gpu_worker(rank, world, port, steps, q):
    """One rank of the gloo-staged rehearsal on one GPU: the device engine on its shard,
    the batched protocol (sharded_reset / scan / resolve / collect), summaries
    exchanged through host copies over gloo (dist.ShardedPlanner(staged=True))."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from kafkabalancer_amd import engine as E
        from kafkabalancer_amd.dist import _DeviceEngineAdapter
        cl, cfg = _gpu_cluster()
        eng = E.Engine(cl, cfg, shard=shard_bounds(cl.n, world, rank))
        sp = ShardedPlanner(_DeviceEngineAdapter(eng), world, device_tensors=True, staged=True)
        out = sp.plan(steps, batch=8)
        q.put((rank, [(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in out],
               eng.state(), None))
        eng.close()
        dist.destroy_process_group()
    except Exception as ex:                        # reported to the parent, not swallowed
        q.put((rank, None, None, repr(ex)))


@pytest.mark.gpu
def test_gloo_two_ranks_gpu_engines_match_oracle():
    """Two processes (gloo, host-staged summaries) running the engine's sharded scan and
    resolve kernels on one GPU: both apply the oracle's plan (oracle/kb_oracle.c)."""
    from kafkabalancer_amd import synth
    from helpers import oracle_plan
    steps = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ch, st, err = q.get(timeout=240)
        assert err is None, "rank %d: %s" % (r, err)
        res[r] = (ch, st)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1]                        # every rank applied the identical plan
    cl, cfg = _gpu_cluster()
    och, oerr, opl = oracle_plan(synth.to_plist(cl), cfg, steps)
    assert oerr is None
    assert res[0][0] == [(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in och]
    assert res[0][1] == opl.state()


@pytest.mark.gpu
def test_sharded_summary_growth_matches_oracle():
    """Exact ties over many broker pairs: more distinct near-tie keys than a 56-key
    (1936-B) rank summary carries.  Every rank halts the step (KB_GROW), the summaries
    grow 8x, the step runs again -- the oracle's plan, no capacity error."""
    from kafkabalancer_amd import engine as E
    from helpers import oracle_plan
    # rings of RF2 partitions in three groups of 20 brokers (unit weights, leader 2,
    # follower 1): every heavy broker carries 12k, every light one 6k, the rest 9k, so
    # all 400 (heavy, light) moves tie; the ring set repeated 12 times (2160 partitions)
    parts = []
    for rep in range(12):
        for g, rings in ((0, 4), (20, 2), (40, 3)):
            for r in range(rings):
                for i in range(20):
                    parts.append({"topic": "t%d" % g, "partition": len(parts),
                                  "replicas": [1 + g + i, 1 + g + (i + 1 + r) % 20]})
    pl = {"version": 1, "partitions": parts}
    cfg = default_cfg(min_unbalance=0.0)
    world, steps = 2, 12
    engs = [E.Engine(pl, cfg, shard=shard_bounds(len(parts), world, r)) for r in range(world)]
    nb0 = engs[0].summary_bytes()
    assert nb0 <= 2048
    got, grows, bufs = [], 0, None
    while len(got) < steps:
        nb = engs[0].summary_bytes()
        if bufs is None or bufs[0].numel() != nb:
            bufs = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
            torch.cuda.synchronize()
        for e, b in zip(engs, bufs):
            e.step_begin(b.data_ptr())
        torch.cuda.synchronize()
        gathered = torch.cat(bufs)
        chs = [e.step_finish(gathered.data_ptr(), world) for e in engs]
        assert chs[0] == chs[1]
        if chs[0] in ("retry", "grow"):
            grows += chs[0] == "grow"
            continue
        if chs[0] is None:
            break
        got.append(chs[0])
    assert grows >= 1 and engs[0].summary_bytes() > nb0
    och, oerr, opl = oracle_plan(pl, cfg, steps)
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert oerr is None
    assert [key(c) for c in got] == [key(c) for c in och]
    assert engs[0].state() == opl.state() == engs[1].state()


def _tie_rings(group, reps, heavy_first=False):
    """RF2 partitions in rings over three groups of `group` brokers (unit weights: the
    leader carries 2, the follower 1): heavy brokers hold 12 per ring set, light ones 6,
    the rest 9, so every (heavy, light) non-leader move ties exactly -- group**2
    distinct near-tie keys.  heavy_first: every heavy-group partition comes first (in
    the first shard), the light and middle groups after them."""
    parts = []
    blocks = {0: [], 1: [], 2: []}
    for rep in range(reps):
        for gi, (g, rings) in enumerate(((0, 4), (group, 2), (2 * group, 3))):
            for r in range(rings):
                for i in range(group):
                    blocks[gi].append([1 + g + i, 1 + g + (i + 1 + r) % group])
    order = blocks[0] + blocks[1] + blocks[2] if heavy_first else \
        [x for rep in zip(blocks[0], blocks[1], blocks[2]) for x in rep]
    for reps_ in order:
        parts.append({"topic": "t", "partition": len(parts), "replicas": reps_})
    return {"version": 1, "partitions": parts}


@pytest.mark.gpu
def test_sharded_summary_capacity_is_the_same_verdict_on_every_rank(monkeypatch):
    """More than SUMMARY_KEYS_MAX (2048) exact-tied keys, all of them on the first shard,
    whose scan spill buffer is also tiny (only that rank spills): the summaries grow
    56 -> 448 -> 2048 keys on both ranks alike, then every rank returns the same
    capacity error -- never one rank KB_GROW while the other errors (which would leave
    the growing rank alone in the next collective)."""
    from kafkabalancer_amd import engine as E
    pl = _tie_rings(50, 3, heavy_first=True)          # 2500 (heavy, light) keys
    cfg = default_cfg(min_unbalance=0.0)
    world = 2
    n = len(pl["partitions"])
    monkeypatch.setenv("KB_CONT_CAP", "4")            # rank 0 only: its spill overflows
    e0 = E.Engine(pl, cfg, shard=shard_bounds(n, world, 0))
    monkeypatch.delenv("KB_CONT_CAP")
    e1 = E.Engine(pl, cfg, shard=shard_bounds(n, world, 1))
    engs = [e0, e1]
    verdicts = []
    for _ in range(16):
        nb = engs[0].summary_bytes()
        assert engs[1].summary_bytes() == nb
        bufs = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(world)]
        torch.cuda.synchronize()
        for e, b in zip(engs, bufs):
            e.step_begin(b.data_ptr())
        torch.cuda.synchronize()
        gathered = torch.cat(bufs)
        out = []
        for e in engs:
            try:
                out.append(e.step_finish(gathered.data_ptr(), world))
            except E.EngineError as ex:
                out.append(("error", ex.args[0] if ex.args else None))
        verdicts.append(out)
        assert out[0] == out[1] or (isinstance(out[0], tuple) and isinstance(out[1], tuple)), out
        if isinstance(out[0], tuple) or out[0] not in ("grow", "retry"):
            break
    last = verdicts[-1]
    assert isinstance(last[0], tuple) and isinstance(last[1], tuple), verdicts
    # 56 -> 448 -> 2048 keys; at 2048 the step runs again while rank 0's spill buffer (the
    # one that overflowed) can still grow -- summary flag bit 2, the same verdict on both
    assert sum(v[0] == "grow" for v in verdicts) >= 2
    for e in engs:
        assert "near-tied candidates in one rank summary" in e.last_error()


def _rccl_worker(steps, port, q):
    """World size 1 over RCCL ("nccl"): the engine on torch's current stream (as
    dist.bench_main sets it up), the batched protocol with all_gather_into_tensor on
    device tensors (ShardedPlanner(staged=False)) -- the driver's multi-GPU path."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        from kafkabalancer_amd import engine as E
        from kafkabalancer_amd.dist import _DeviceEngineAdapter
        cl, cfg = _gpu_cluster()
        eng = E.Engine(cl, cfg, shard=shard_bounds(cl.n, 1, 0))
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        sp = ShardedPlanner(_DeviceEngineAdapter(eng), 1, device_tensors=True, staged=False)
        out = sp.plan(steps, batch=8)
        out += [c for c in [sp.step()] if c is not None]       # the per-step protocol once
        q.put(([(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in out],
               eng.state(), dist.get_backend(), None))
        eng.close()
        dist.destroy_process_group()
    except Exception as ex:                        # reported to the parent, not swallowed
        q.put((None, None, None, repr(ex)))


@pytest.mark.gpu
def test_rccl_world1_matches_oracle():
    """The RCCL exchange path itself: one child process (started before it
    touches the GPU) with init_process_group("nccl"), the engine on torch's stream and
    all_gather_into_tensor between scan and resolve; the oracle's plan."""
    from kafkabalancer_amd import synth
    from helpers import oracle_plan
    steps = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(steps, _free_port(), q))
    p.start()
    ch, st, backend, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert backend == "nccl"
    cl, cfg = _gpu_cluster()
    och, oerr, opl = oracle_plan(synth.to_plist(cl), cfg, steps + 1)
    assert oerr is None
    assert ch == [(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in och]
    assert st == opl.state()


def _rccl_c_worker(steps, q):
    """kb_engine_sharded_plan at world size 1: the RCCL communicator bound by the engine
    itself (kb_comm_unique_id / kb_engine_comm_init), the whole plan driven from C."""
    try:
        torch.cuda.set_device(0)
        from kafkabalancer_amd import engine as E
        cl, cfg = _gpu_cluster()
        uid = E.comm_unique_id()
        eng = E.Engine(cl, cfg, shard=shard_bounds(cl.n, 1, 0))
        eng.comm_init(1, 0, uid)
        a, err = eng.sharded_plan(10)                 # two calls: the plan resumes
        assert err is None, err
        b, err = eng.sharded_plan(steps - 10)
        assert err is None, err
        q.put(([(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in a + b],
               eng.state(), None))
        eng.close()
    except Exception as ex:                        # reported to the parent, not swallowed
        q.put((None, None, repr(ex)))


@pytest.mark.gpu
def test_rccl_sharded_plan_from_c_matches_oracle():
    """The RCCL path driven from C (kb_engine_sharded_plan: scan + summary, ncclAllGather on
    the engine's stream, resolve; 64 rounds per host round trip) equals the oracle's plan
    and final state, in a child process started before it touches the GPU."""
    from kafkabalancer_amd import synth
    from helpers import oracle_plan
    steps = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_c_worker, args=(steps, q))
    p.start()
    ch, st, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    cl, cfg = _gpu_cluster()
    och, oerr, opl = oracle_plan(synth.to_plist(cl), cfg, steps)
    assert oerr is None
    assert ch == [(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in och]
    assert st == opl.state()


def _rccl_wide_worker(steps, q):
    """A world-1 sharded plan at 2500 brokers (the tightening bound pass on every scan)
    next to the plain plan of the same cluster, in one child process."""
    try:
        torch.cuda.set_device(0)
        from kafkabalancer_amd import engine as E
        from kafkabalancer_amd import synth
        cl = synth.make_cluster(20000, 2500, 3, "zipf", seed=0x5EED00B5)
        cfg = {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2, "min_unbalance": 0.0,
               "brokers": None}
        uid = E.comm_unique_id()
        eng = E.Engine(cl, cfg, shard=shard_bounds(cl.n, 1, 0))
        eng.comm_init(1, 0, uid)
        a, err = eng.sharded_plan(steps)
        assert err is None, err
        sh = ([(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in a], eng.state(),
              eng.stats()["spill_grows"])
        eng.close()
        ref = E.Engine(cl, cfg)
        b, err = ref.plan(steps)
        assert err is None, err
        pl = ([(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]) for c in b], ref.state())
        ref.close()
        q.put((sh, pl, None))
    except Exception as ex:                        # reported to the parent, not swallowed
        q.put((None, None, repr(ex)))


@pytest.mark.gpu
def test_rccl_sharded_plan_wide_brokers_matches_plain():
    """Sharded engines at B >= 2048 run the tightening bound pass before every scan (a rank's
    bound from its one gathered summary is open or loose there, and the census spilled
    every wave: c5 0.2 s per step): same plan and state as the plain engine, no spill
    growth."""
    steps = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_wide_worker, args=(steps, q))
    p.start()
    sh, pl, err = q.get(timeout=300)
    p.join(timeout=60)
    assert err is None, err
    assert len(sh[0]) == steps
    assert sh[0] == pl[0]
    assert sh[1] == pl[1]
    assert sh[2] == 0


@pytest.mark.gpu
def test_bench_sharded_world1_line():
    """`bench.py --sharded`: the world-1 sharded protocol line, with the sharded plan equal
    to the plain plan over the same steps."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--sharded", "--workload", "c3",
                        "--scale", "0.05", "--steps", "40", "--warmup", "5"],
                       cwd=root, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["plans_equal"] and line["steps"] == 40, line


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks(tmp_path):
    """`bench.py --gpus 2` with no launcher starts two ranks itself (torch.distributed.run as
    a child process, before any GPU call in the parent); KB_DIST_BACKEND=gloo lets both
    ranks share the box's one GPU.  The line says n_gpus 2, and the timed plan of the
    strong-scaled (one cluster, two shards) run equals one engine's plan of the same steps."""
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "plan.json"
    env = dict(os.environ, KB_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "c3",
                        "--scale", "0.02", "--scaling", "strong", "--steps", "30", "--warmup", "5",
                        "--no-cpu-baseline", "--plan-out", str(out)],
                       cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong", line
    got = json.load(open(out))
    cl, cfg, _ = synth.config("c3", scale=0.02)
    eng = E.Engine(cl, cfg)
    want, err = eng.plan(35)
    assert err is None
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert [key(c) for c in got] == [key(c) for c in want[5:35]]
    eng.close()


@pytest.mark.gpu
def test_bench_main_rccl_world1(tmp_path):
    """The multi-GPU bench path with RCCL (its default backend) under a one-rank
    torch.distributed.run launch: both engines it builds (the timed plan and the kernel-timing
    replay) get communicators of their own unique ids, the line is printed, and the plan
    equals one engine's plan of the same steps."""
    import socket
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "plan.json"
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.pop("KB_DIST_BACKEND", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(root, "bench.py"), "--dist-world1", "--workload", "c3", "--scale", "0.02",
                        "--steps", "30", "--warmup", "5", "--no-cpu-baseline", "--plan-out", str(out)],
                       cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["exchange"] == "rccl" and line["scaling"] == "strong", line
    assert line["roofline"]["avg_launch_us"] > 0 and 0 < line["roofline"]["frac"] < 1, line["roofline"]
    got = json.load(open(out))
    cl, cfg, _ = synth.config("c3", scale=0.02)
    eng = E.Engine(cl, cfg)
    want, err = eng.plan(35)
    assert err is None
    key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
    assert [key(c) for c in got] == [key(c) for c in want[5:35]]
    eng.close()
