"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bit-exact bar: identical change sequences (step, partition, kind, from, to,
slot), identical final replica state and broker loads, identical error
messages; unbalance values within 1e-9 relative (BASELINE.json north_star).
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O
from kafkabalancer_amd import engine as E
from kafkabalancer_amd import synth

from test_gpu_parity_data import random_plist
from helpers import (assert_same_plan, default_cfg, golden, oracle_loads, oracle_plan, rel_close)

pytestmark = pytest.mark.gpu

SEM = {"applied": (E.KB_SEM_APPLIED, O.SEM_APPLIED), "go": (E.KB_SEM_GO, O.SEM_GO)}


def engine_plan(plist_or_cluster, cfg, steps, sem="applied"):
    eng = E.Engine(plist_or_cluster, cfg, semantics=SEM[sem][0])
    changes, err = eng.plan(steps)
    return eng, changes, err


def check_plan(plist, cfg, steps, sem="applied"):
    eng, ech, eerr = engine_plan(plist, cfg, steps, sem)
    och, oerr, opl = oracle_plan(plist, cfg, steps, SEM[sem][1])
    assert_same_plan(ech, eerr, och, oerr)
    if oerr is None:
        assert eng.state() == opl.state()
        if sem == "applied" and plist["partitions"]:
            st = opl.state()
            ws = [opl.partition(i)["weight"] for i in range(opl.n)]
            ncs = [opl.partition(i)["num_consumers"] for i in range(opl.n)]
            want = oracle_loads(st, ws, ncs)
            got = eng.loads()
            for b, l in want.items():
                assert got[b] == l, (b, got[b], l)
    eng.close()
    return ech


# ------------------------------------------------------------ golden cases

def test_balancer_golden_cases():
    g = golden("balancer_cases.json")
    for c in g["cases"]:
        cfg = default_cfg(**g["configs"][c["cfg"]])
        pl = {"version": 1, "partitions": c["pl"]}
        eng = E.Engine(pl, cfg, semantics=E.KB_SEM_APPLIED)
        if "err" in c:
            with pytest.raises(E.EngineError) as ei:
                eng.balance()
            assert c["err"] in str(ei.value), (c["line"], str(ei.value))
            # the exact reference message, as the oracle formats it
            r = O.balance(O.OraclePL(pl), cfg)
            assert str(ei.value) == r["err"]
        elif c["ppl"] is None:
            assert eng.balance() is None, c["line"]
        else:
            ch = eng.balance()
            exp = c["ppl"][0]
            got_p = pl["partitions"][ch["pidx"]]
            assert (got_p["topic"], got_p["partition"]) == (exp["topic"], exp["partition"]), c["line"]
            assert eng.replicas(ch["pidx"]) == exp["replicas"], c["line"]
        eng.close()


def test_balancer_golden_cases_go_semantics():
    g = golden("balancer_cases.json")
    for c in g["cases"]:
        cfg = default_cfg(**g["configs"][c["cfg"]])
        pl = {"version": 1, "partitions": c["pl"]}
        check_plan(pl, cfg, 3, "go")


# ------------------------------------------------------------- c1 plans

@pytest.mark.parametrize("sem", ["applied", "go"])
@pytest.mark.parametrize("variant", ["default", "leader", "rebalance", "brokers", "min1", "min0unb"])
def test_c1_plans(variant, sem):
    pl = golden("test.json")
    cfg = default_cfg()
    if variant == "leader":
        cfg["allow_leader"] = True
    elif variant == "rebalance":
        cfg["rebalance_leaders"] = True
        cfg["min_unbalance"] = 0.0
    elif variant == "brokers":
        cfg["brokers"] = [1, 2, 3, 4, 5, 6]
    elif variant == "min1":
        cfg["min_replicas"] = 1
        cfg["allow_leader"] = True
    elif variant == "min0unb":
        cfg["min_unbalance"] = 0.0
    check_plan(pl, cfg, 40, sem)


def test_c1_golden_plans():
    """The committed golden plans (tests/golden/plans_small.json) replayed on the GPU."""
    g = golden("plans_small.json")
    for case in g["cases"]:
        sem = case["sem"]
        eng, ech, eerr = engine_plan(case["plist"], case["cfg"], case["steps"], sem)
        got = [[c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]] for c in ech]
        assert got == case["changes"], case["name"]
        assert (eerr is None) == (case["err"] is None), (case["name"], eerr, case["err"])
        if case["err"] is not None and ": panic" not in case["err"]:
            assert str(eerr) == case["err"]
        assert eng.state() == case["final"], case["name"]
        eng.close()


# ------------------------------------------------------ random small cases

CASES = []
for seed in range(40):
    r = random.Random(seed)
    CASES.append(dict(seed=seed, P=r.choice([3, 8, 20, 60, 150]), B=r.choice([2, 3, 4, 6, 10, 25]),
                      weights=r.choice(["uniform", "int", "zipf"]), sets=r.choice(["none", "some", "all"]),
                      nrvar=r.random() < 0.4, ncons=r.random() < 0.3,
                      allow_leader=r.random() < 0.5, rebalance=r.random() < 0.25,
                      min_replicas=r.choice([1, 2, 2, 3]), min_unbalance=r.choice([0.0, 0.0, 0.01, 1e-6]),
                      explicit=r.random() < 0.25, sem=r.choice(["applied", "applied", "go"])))


@pytest.mark.parametrize("case", CASES, ids=lambda c: "s%d" % c["seed"])
def test_random_small(case):
    rng = random.Random(1000 + case["seed"])
    pl = random_plist(rng, case["P"], case["B"], case["weights"], case["sets"], case["nrvar"], case["ncons"])
    cfg = default_cfg(allow_leader=case["allow_leader"], rebalance_leaders=case["rebalance"],
                      min_replicas=case["min_replicas"], min_unbalance=case["min_unbalance"])
    if case["explicit"]:
        cfg["brokers"] = list(range(1, case["B"] + 3))
    check_plan(pl, cfg, 30, case["sem"])


# ------------------------------------------------- BASELINE configs (scaled)

def test_c2_full_plan():
    """configs[1]: 10k partitions x 50 brokers, RF3, uniform weights, 100-move plan."""
    cl, cfg, _ = synth.config("c2", with_names=True)
    pl = synth.to_plist(cl)
    ech = check_plan(pl, cfg, 100)
    assert len(ech) == 100


def test_spill_growth_matches_oracle(monkeypatch):
    """Exact ties overflowing the near-tie spill buffer (a 4-candidate buffer here,
    KB_CONT_CAP): the host grows it and the step runs again -- same plan as the oracle,
    no capacity error."""
    monkeypatch.setenv("KB_CONT_CAP", "4")
    # three groups of 20 brokers in rings of RF2 partitions (leader 2, follower 1 with
    # unit weights): every heavy broker carries 12, every light one 6, the rest 9, so
    # all 400 (heavy, light) moves tie and the census collects far more keys than a
    # scan workgroup record holds
    parts = []
    for g, rings in ((0, 4), (20, 2), (40, 3)):
        for r in range(rings):
            for i in range(20):
                parts.append({"topic": "t%d" % g, "partition": len(parts),
                              "replicas": [1 + g + i, 1 + g + (i + 1 + r) % 20]})
    pl = {"version": 1, "partitions": parts}
    cfg = default_cfg(min_unbalance=0.0)
    eng = E.Engine(pl, cfg)
    ech, eerr = eng.plan(25)
    och, oerr, opl = oracle_plan(pl, cfg, 25)
    assert_same_plan(ech, eerr, och, oerr)
    assert eng.state() == opl.state()
    assert eng.stats()["spill_grows"] >= 1
    eng.close()


@pytest.mark.parametrize("variant", ["c3", "c4"])
def test_scaled_configs(variant):
    if variant == "c3":
        cl = synth.make_cluster(6000, 300, 3, "zipf", nsets=24, set_size=32, seed=11, with_names=True)
        cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
    else:
        nr = np.zeros(6000, np.int64)
        nr[[5, 900, 3000]] = 2
        nr[[7, 1500, 4500]] = 4
        cl = synth.make_cluster(6000, 300, 3, "zipf", seed=12, with_names=True, num_replicas=nr)
        cfg = default_cfg(min_unbalance=0.0, brokers=[b for b in range(1, 361) if not 280 <= b <= 300])
    pl = synth.to_plist(cl)
    check_plan(pl, cfg, 12)


@pytest.mark.parametrize("allow_leader", [False, True])
def test_stage_transition_into_move(allow_leader):
    """RemoveExtraReplicas / AddMissingReplicas steps, then move(): the scans after a
    first-index stage skip the near-tie census (ub = -inf) and the first move() step
    re-scans with the bound opened (k_step retry); the plan must not notice."""
    nr = np.zeros(2000, np.int64)
    nr[[11, 700]] = 2
    nr[[5, 1300, 1999]] = 4
    cl = synth.make_cluster(2000, 40, 3, "zipf", seed=41, with_names=True, num_replicas=nr)
    cfg = default_cfg(allow_leader=allow_leader, min_unbalance=0.0)
    pl = synth.to_plist(cl)
    ech = check_plan(pl, cfg, 12)
    steps = [c["step"] for c in ech]
    assert steps[:5] == ["RemoveExtraReplicas"] * 2 + ["AddMissingReplicas"] * 3
    assert all(s in ("MoveLeaders", "MoveNonLeaders") for s in steps[5:]) and len(steps) == 12


def test_many_brokers_sorting():
    """4096-entry broker table (c5 width) with explicit broker ids, tiny P for the oracle."""
    cl = synth.make_cluster(120, 4096, 3, "int", seed=5, with_names=True)
    cfg = default_cfg(min_unbalance=0.0, brokers=list(range(1, 4097)))
    pl = synth.to_plist(cl)
    check_plan(pl, cfg, 2)


def test_broker_tables_in_memory_literal_oracle():
    """Past the 4096 brokers the kernels keep in LDS the broker tables live in memory
    (k_scan's GT and k_step's GB instantiations): 5000 listed brokers, tiny P for the
    literal oracle loop (threaded; the scale_b6000 / b8000 / b12000 / b16384 fixtures of
    test_golden_scale.py cover the larger cases)."""
    cl = synth.make_cluster(60, 5000, 3, "int", seed=7, with_names=True, broker_hi=5000)
    cfg = default_cfg(min_unbalance=0.0, brokers=list(range(1, 5001)))
    pl = synth.to_plist(cl)
    O.set_threads(min(16, os.cpu_count() or 1))
    try:
        check_plan(pl, cfg, 3)
    finally:
        O.set_threads(1)


# ------------------------------------------ full-size properties (c3 size)

def test_full_size_properties():
    cl, cfg, _ = synth.config("c3")
    eng = E.Engine(cl, cfg)
    ch1, err = eng.plan(40)
    assert err is None and len(ch1) == 40
    # determinism: a second engine on the same input produces the identical plan
    eng2 = E.Engine(cl, cfg)
    ch2, _ = eng2.plan(40)
    assert [tuple(sorted(c.items())) for c in ch1] == [tuple(sorted(c.items())) for c in ch2]
    # loads stay the exact partition-ordered fold (getBrokerLoad, utils.go:92-105) of
    # the replayed final state
    got = eng.loads()
    reps = cl.replica_ids.reshape(-1, 3).copy()
    for c in ch1:
        row = reps[c["pidx"]]
        row[c["slot"]] = c["to"]
    want = oracle_loads(reps.tolist(), cl.weight.tolist(), [0] * cl.n)
    for b, l in want.items():
        assert got[b] == l, (b, got[b], l)
    # the engine's unbalance is the oracle's getUnbalanceBL fold (utils.go:119-147) of
    # those loads in getBL order (utils.go:107-117), bit for bit
    bl = sorted(want.items(), key=lambda kv: (kv[1], kv[0]))
    u_exact = O.unbalance(np.array([l for _, l in bl]))
    assert eng.unbalance() == u_exact
    # and the next step starts from it: su of step 41 is that fold (exact, or within 1e-9)
    ch3, err = eng.plan(1)
    assert err is None and len(ch3) == 1
    if ch3[0]["exact"]:
        assert ch3[0]["su"] == u_exact
    assert rel_close(ch3[0]["su"], u_exact)
    eng.close()
    eng2.close()


def test_distribute_leaders_empty_partition_after_pick():
    """distributeLeaders builds pp over every partition (steps.go:257-262): an empty
    Replicas anywhere panics, even after an eligible heavy-leader partition."""
    from test_oracle import EMPTY_AFTER_PICK
    for sem in ("applied", "go"):
        check_plan(EMPTY_AFTER_PICK, default_cfg(rebalance_leaders=True, min_unbalance=0.0), 3, sem)
        check_plan(EMPTY_AFTER_PICK, default_cfg(min_unbalance=0.0), 3, sem)


# ------------------------------------- lower-bound prune of the scan (k_scan)

def _plan_with_scan_dbg(cl, cfg, steps, dbg):
    old = os.environ.get("KB_DEBUG_SCAN")
    os.environ["KB_DEBUG_SCAN"] = str(dbg)
    try:
        eng = E.Engine(cl, cfg)
    finally:
        if old is None:
            del os.environ["KB_DEBUG_SCAN"]
        else:
            os.environ["KB_DEBUG_SCAN"] = old
    ch, err = eng.plan(steps)
    st = eng.stats()
    eng.close()
    return ch, err, st


@pytest.mark.parametrize("variant", ["c3", "c2", "c4s"])
def test_scan_prune_invariant(variant):
    """The prune (waves whose lower bound is above ub + 16 eps only count their
    candidates) changes neither the plan nor the candidate count: same run with the
    prune disabled (KB_DEBUG_SCAN=16)."""
    if variant == "c3":
        cl, cfg, _ = synth.config("c3")
        steps = 60
    elif variant == "c2":
        cl, cfg, _ = synth.config("c2")
        steps = 100
    else:
        nr = np.zeros(200000, np.int64)
        nr[[5, 90000, 150000]] = 2
        nr[[7, 100000, 190000]] = 4
        cl = synth.make_cluster(200000, 400, 3, "zipf", nsets=64, set_size=48, seed=21, num_replicas=nr)
        cfg = default_cfg(allow_leader=True, min_unbalance=0.0, brokers=list(range(1, 451)))
        steps = 40
    ch1, e1, s1 = _plan_with_scan_dbg(cl, cfg, steps, 0)
    ch0, e0, s0 = _plan_with_scan_dbg(cl, cfg, steps, 16)
    assert e1 == e0
    assert [tuple(sorted(c.items())) for c in ch1] == [tuple(sorted(c.items())) for c in ch0]
    assert s1["candidates"] == s0["candidates"] > 0


def test_candidate_count_first_step():
    """Metric 1 on the first step, counted independently in numpy:
    sum over eligible partitions of |allowed ∩ bl| - |replicas ∩ allowed| per
    non-leader slot (steps.go:167-201; no leader step without -allow-leader)."""
    cl = synth.make_cluster(300000, 500, 3, "zipf", nsets=40, set_size=64, seed=33)
    cfg = default_cfg(min_unbalance=0.0)
    eng = E.Engine(cl, cfg)
    ch, err = eng.plan(1)
    assert err is None and len(ch) == 1
    cand = eng.stats()["candidates"]
    eng.close()
    reps = cl.replica_ids.reshape(-1, 3)
    present = np.zeros(int(reps.max()) + 2, bool)
    present[reps.reshape(-1)] = True
    want = 0
    for s in range(len(cl.set_off) - 1):
        members = cl.set_ids[cl.set_off[s]:cl.set_off[s + 1]]
        inset = np.zeros_like(present)
        inset[members] = True
        n_elig = int((present & inset).sum())
        rows = reps[cl.set_idx == s]
        nin = inset[rows].sum(axis=1)
        want += int(((n_elig - nin) * 2).sum())
    assert cand == want


# ------------------------------------------------- many distinct broker lists
# More distinct `Brokers` lists than the meta word's 15-bit set field holds (and than
# fit in LDS): the scan reads the per-partition set index array and the set records
# from memory, k_step rebuilds the records from list-driven chunks (utils.go:66-90,
# steps.go:117-143; the reference has no such limit).

def _many_sets_plist(seed, P, B, disallowed=0.0, nrvar=0.0):
    rng = random.Random(seed)
    parts = []
    for i in range(P):
        reps = rng.sample(range(1, B + 1), 3)
        extra = rng.sample([b for b in range(1, B + 1) if b not in reps], rng.randint(2, 5))
        allowed = list(reps) + extra
        if disallowed and rng.random() < disallowed:
            allowed.remove(reps[rng.randint(0, 2)])      # a replica outside the list
        p = {"topic": "t%d" % (i % 5), "partition": i, "replicas": reps,
             "weight": rng.uniform(1, 1e6) ** -1.1, "brokers": sorted(allowed)}
        if nrvar and rng.random() < nrvar:
            p["num_replicas"] = rng.choice([2, 4])
        parts.append(p)
    return {"version": 1, "partitions": parts}


@pytest.mark.parametrize("variant", ["moves", "disallowed", "add_remove"])
def test_many_distinct_broker_lists(variant):
    P, B = 100_000, 200
    pl = _many_sets_plist(7, P, B, disallowed=0.0005 if variant == "disallowed" else 0.0,
                          nrvar=0.0003 if variant == "add_remove" else 0.0)
    nsets = len({tuple(p["brokers"]) for p in pl["partitions"]})
    assert nsets > 90_000, nsets                     # past the 15-bit field (32767) and LDS
    cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
    ech = check_plan(pl, cfg, 25)
    assert len(ech) == 25
    if variant == "disallowed":
        assert any(c["step"] == "MoveDisallowedReplicas" for c in ech)
    if variant == "add_remove":
        assert {"RemoveExtraReplicas", "AddMissingReplicas"} & {c["step"] for c in ech}
