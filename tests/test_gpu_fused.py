"""The fused pair (k_pair: the scan's grid plus one resident step workgroup per launch)
against the two-launch pair (k_scan + k_step, KB_FUSE=0): the same plans, the same device
state after them (every broker load bit for bit), on the headline shape, on c5's broker
width with eager refolds and fold checkpoints, and the small-shard gate (c2 keeps two
launches).  The parity of both against the oracle is the rest of the -m gpu suite."""
import os

import pytest

from kafkabalancer_amd import engine as E
from kafkabalancer_amd import synth

pytestmark = pytest.mark.gpu


def run(cl, cfg, steps, fuse):
    old = os.environ.get("KB_FUSE")
    os.environ["KB_FUSE"] = "1" if fuse else "0"
    try:
        eng = E.Engine(cl, cfg)
    finally:
        if old is None:
            del os.environ["KB_FUSE"]
        else:
            os.environ["KB_FUSE"] = old
    changes, err = eng.plan(steps)
    st = eng.stats()
    loads = eng.loads()
    eng.close()
    return changes, err, st, loads


def keyed(changes):
    return [(c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"], c["su"], c["cu"]) for c in changes]


# (full size: the pair is fused only when the scan tiles are full -- 16 scoring waves)
@pytest.mark.parametrize("name,scale,steps", [("c3", 1.0, 200), ("c4", 1.0, 400)])
def test_fused_matches_two_launches(name, scale, steps):
    cl, cfg, _ = synth.config(name, scale=scale)
    a = run(cl, cfg, steps, True)
    b = run(cl, cfg, steps, False)
    assert a[2]["fused_pairs"] == 1 and b[2]["fused_pairs"] == 0
    assert (a[1] is None) == (b[1] is None)
    assert keyed(a[0]) == keyed(b[0])
    assert a[3] == b[3]


def test_fused_eager_checkpoints_match_two_launches():
    """c5's broker width (1M partitions x 4096 brokers, Zipf): eager refolds with fold
    checkpoints inside the fused launch, against the two-launch pair."""
    cl = synth.make_cluster(1_000_000, 4096, 3, "zipf", seed=0x5EED5005)
    cfg = {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2, "min_unbalance": 0.0,
           "brokers": None}
    a = run(cl, cfg, 80, True)
    b = run(cl, cfg, 80, False)
    assert a[2]["fused_pairs"] == 1
    assert keyed(a[0]) == keyed(b[0])
    assert a[3] == b[3]


def _with_env(name, value, fn):
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        return fn()
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


def test_small_shard_fused_matches_two_launches():
    """c2's 10k partitions (79 scan workgroups of one scoring wave) run as fused pairs since
    round 6 (the fast / deferred prep exists only in the fused step); the plan, every
    unbalance figure and the final state equal the two-launch path's (KB_FUSE_SMALL=0)."""
    cl, cfg, _ = synth.config("c2")
    out = []
    for v in ("1", "0"):
        eng = _with_env("KB_FUSE_SMALL", v, lambda: E.Engine(cl, cfg))
        ch, err = eng.plan(100)
        assert err is None, err
        out.append((eng.stats()["fused_pairs"], ch, eng.state()))
        eng.close()
    (f1, c1, s1), (f0, c0, s0) = out
    assert f1 == 1 and f0 == 0, (f1, f0)
    assert len(c1) == 100
    assert c1 == c0
    assert s1 == s0


def test_pair_timeout_poisons_engine():
    """k_pair's step workgroup gives up waiting for its grid (forced: a zero wait bound):
    the plan stops with the explicit error, the arrival count is reset once the stream is
    idle, and the engine refuses further plans; a new engine then plans normally."""
    cl, cfg, _ = synth.config("c3", scale=1.0)          # (fused only with full scan tiles)
    eng = _with_env("KB_PAIR_WAIT_TICKS", "0", lambda: E.Engine(cl, cfg))
    assert eng.stats()["fused_pairs"] == 1
    changes, err = eng.plan(5)
    assert err is not None and "timed out" in str(err), err
    changes, err = eng.plan(5)
    assert changes == [] and err is not None and "unusable" in str(err), err
    with pytest.raises(E.EngineError) as ei:
        eng.balance()
    assert "unusable" in str(ei.value)
    eng.close()
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(20)
    assert err is None and len(want) == 20
    ref.close()


@pytest.mark.parametrize("mode", ["0", "1"])
def test_control_transfer_modes_match(mode):
    """The batch-end control-block / log transfer (k_xfer polled by the host, the default)
    against a k_xfer with a stream synchronisation and hipMemcpyAsync (KB_XFER=1 / 0): the
    same plans and loads bit for bit, across several batches and kb_engine_balance calls."""
    cl, cfg, _ = synth.config("c3", scale=1.0)
    a = run(cl, cfg, 150, True)
    b = _with_env("KB_XFER", mode, lambda: run(cl, cfg, 150, True))
    assert keyed(a[0]) == keyed(b[0])
    assert a[3] == b[3]
    eng = _with_env("KB_XFER", mode, lambda: E.Engine(cl, cfg))
    ref = E.Engine(cl, cfg)
    for _ in range(5):
        assert keyed([eng.balance()]) == keyed([ref.balance()])
    eng.close()
    ref.close()


class _DevBuf:
    """A zeroed device buffer from the HIP runtime the engine uses (no torch: only the
    engine's own stream touches it)."""
    _hip = None

    def __init__(self, nbytes):
        import ctypes
        if _DevBuf._hip is None:
            _DevBuf._hip = ctypes.CDLL("libamdhip64.so")
        self.p = ctypes.c_void_p()
        assert _DevBuf._hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(nbytes)) == 0
        assert _DevBuf._hip.hipMemset(self.p, 0, ctypes.c_size_t(nbytes)) == 0
        assert _DevBuf._hip.hipDeviceSynchronize() == 0

    def ptr(self):
        return self.p.value

    def free(self):
        _DevBuf._hip.hipFree(self.p)


def _sharded_world1(cl, cfg, steps, env):
    """The batched sharded protocol at world size 1 (the summary is its own gathered
    buffer), with the given environment at engine creation; (changes, error, stats, loads)."""
    eng = _with_env(*env, lambda: E.Engine(cl, cfg, shard=(0, cl.n)))
    got, err, bufs = [], None, []
    try:
        done = False
        while not done and len(got) < steps:
            summ = _DevBuf(eng.summary_bytes())
            bufs.append(summ)
            batch = min(16, steps - len(got))
            eng.sharded_reset(batch)
            for _ in range(batch):
                eng.sharded_scan(summ.ptr())
                eng.sharded_resolve(summ.ptr(), 1)
            st, ch = eng.sharded_collect(batch + 1)
            got.extend(ch)
            done = st == "done"
    except E.EngineError as ex:
        err = ex
    st = eng.stats()
    loads = eng.loads() if err is None else None
    eng.close()
    for b in bufs:
        b.free()
    return got, err, st, loads


@pytest.mark.parametrize("allow_leader", [True, False])
def test_fused_summary_matches_two_launches(allow_leader):
    """k_scansum (the rank summary in the scan's grid) against k_scan + k_summary: the same
    sharded plan and final loads, with and without -allow-leader (the BK instantiation)."""
    cl, cfg, _ = synth.config("c3", scale=0.25)
    cfg = dict(cfg, allow_leader=allow_leader)
    a = _sharded_world1(cl, cfg, 60, ("KB_FUSE_SUM", "1"))
    b = _sharded_world1(cl, cfg, 60, ("KB_FUSE_SUM", "0"))
    assert a[2]["fused_summaries"] == 1 and b[2]["fused_summaries"] == 0
    assert a[1] is None and b[1] is None
    assert len(a[0]) == 60
    assert keyed(a[0]) == keyed(b[0])
    assert a[3] == b[3]


def test_summary_timeout_poisons_engine():
    """k_scansum's summary workgroup gives up waiting for its grid (a zero wait bound): the
    batch ends with the explicit error, the arrival count is reset, and the engine refuses
    further sharded work."""
    cl, cfg, _ = synth.config("c3", scale=0.25)
    eng = _with_env("KB_PAIR_WAIT_TICKS", "0", lambda: E.Engine(cl, cfg, shard=(0, cl.n)))
    assert eng.stats()["fused_summaries"] == 1
    summ = _DevBuf(eng.summary_bytes())
    eng.sharded_reset(4)
    for _ in range(4):
        eng.sharded_scan(summ.ptr())
        eng.sharded_resolve(summ.ptr(), 1)
    with pytest.raises(E.EngineError) as ei:
        eng.sharded_collect(5)
    assert "timed out" in str(ei.value)
    with pytest.raises(E.EngineError) as ei:
        eng.sharded_reset(1)
    assert "unusable" in str(ei.value)
    eng.close()
    summ.free()
    got, err, st, _ = _sharded_world1(cl, cfg, 10, ("KB_FUSE_SUM", "1"))
    assert err is None and len(got) == 10 and st["fused_summaries"] == 1


def test_sharded_summary_wide_brokers_match_plain_plan():
    """A sharded engine past SUM_RLDS brokers (9000: broker tables in memory, k_summary
    re-scores the keys from r in memory, no fused summary) gives the unsharded plan."""
    cl = synth.make_cluster(30000, 9000, 3, "zipf", seed=0x5EED9000)
    cfg = {"allow_leader": True, "rebalance_leaders": False, "min_replicas": 2, "min_unbalance": 0.0,
           "brokers": None}
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(24)
    ref.close()
    assert err is None and len(want) == 24
    got, err, st, _ = _sharded_world1(cl, cfg, 24, ("KB_FUSE_SUM", "1"))
    assert err is None and st["fused_summaries"] == 0
    assert keyed(got) == keyed(want)


def test_torch_hip_init_after_engine_sharded():
    """A host that initialises HIP through torch only after kb_engine_create (the pattern
    commit 43f2c44 moved the world-1 sharded tests away from): torch's first CUDA tensor
    comes after the engine's HIP state, and the batched sharded protocol then runs over that
    torch buffer.  The plan must equal the one over a hipMalloc'd buffer, which the tests
    above use.  (Run in a child process so that torch's CUDA state starts uninitialised.)"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import json, sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import torch
from kafkabalancer_amd import engine as E
from kafkabalancer_amd import synth
import test_gpu_fused as T
cl, cfg, _ = synth.config("c3", scale=0.05)
eng = E.Engine(cl, cfg, shard=(0, cl.n))           # engine HIP state first
assert not torch.cuda.is_initialized()
summ = torch.zeros(eng.summary_bytes(), dtype=torch.uint8, device="cuda")   # then torch's
torch.cuda.synchronize()
got = []
while len(got) < 30:
    eng.sharded_reset(10)
    for _ in range(10):
        eng.sharded_scan(summ.data_ptr())
        eng.sharded_resolve(summ.data_ptr(), 1)
    st, ch = eng.sharded_collect(11)
    got.extend(ch)
    if st == "done":
        break
eng.close()
ref, err, _, _ = T._sharded_world1(cl, cfg, 30, ("KB_FUSE_SUM", "1"))
key = lambda c: (c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"])
print(json.dumps({"n": len(got), "equal": [key(c) for c in got[:30]] == [key(c) for c in ref[:30]],
                  "err": None if err is None else str(err)}))
''' % (root, os.path.join(root, "tests"))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["err"] is None and res["n"] >= 30 and res["equal"], res


def _run_env(cl, cfg, steps, env):
    eng = _with_env(*env, lambda: E.Engine(cl, cfg))
    changes, err = eng.plan(steps)
    st = eng.stats()
    loads = eng.loads()
    eng.close()
    return changes, err, st, loads


# (full size: the pair is fused at full tiles; c3 -- the headline's leader 2-cycle -- and c3nl
# -- a different partition almost every step)
@pytest.mark.parametrize("name,allow_leader,steps", [("c3", True, 300), ("c3", False, 300)])
def test_fast_prep_matches_full_prep(name, allow_leader, steps):
    """The deferred prep (DevCtl.fp: the order, the positions and the set records of a plain
    move left to the next launch's step workgroup, the scan patching the positions) gives the
    plans and the device state of the full prep every step (KB_FP=0): every change with its
    su / cu bits, every broker load; and it is the path the plan took."""
    cl, cfg, _ = synth.config(name, scale=1.0)
    cfg = dict(cfg, allow_leader=allow_leader)
    a = _run_env(cl, cfg, steps, ("KB_FP", "1"))
    b = _run_env(cl, cfg, steps, ("KB_FP", "0"))
    assert a[1] is None and b[1] is None
    assert keyed(a[0]) == keyed(b[0])
    assert a[3] == b[3]
    assert a[2]["fast_preps"] > steps // 2 and b[2]["fast_preps"] == 0, (a[2]["fast_preps"], b[2]["fast_preps"])
