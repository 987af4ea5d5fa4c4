"""The per-step boundary (kb_engine_step): one Balance() restricted to a
subset of the reference's steps table (balancer.go:34-44), so a host that keeps the
reference's table and Balance() binds each entry to one call.

Checked against the oracle's or_step (the same Balance() over the same subset of steps,
steps.go:7-307):
  * the steps table walked on the host, one call per entry, equals the fused pipeline
    (kb_engine_plan) and the oracle's Balance() sequence;
  * single steps called on their own (MoveNonLeaders alone while partitions still hold
    disallowed replicas or extra replicas, RemoveExtraReplicas alone, ...) equal the
    oracle's step function called on its own;
  * random mask sequences, both semantics;
  * at scale (c3's shape): the table walk reuses the scan of a step that changed nothing
    and still equals the device-resident plan.
"""
import random

import pytest

from oracle import oracle as O
from kafkabalancer_amd import engine as E
from kafkabalancer_amd import synth

from test_gpu_parity_data import random_plist
from helpers import assert_same_plan, default_cfg, golden, oracle_loads

pytestmark = pytest.mark.gpu

SEM = {"applied": (E.KB_SEM_APPLIED, O.SEM_APPLIED), "go": (E.KB_SEM_GO, O.SEM_GO)}
BIT = {n: 1 << i for i, n in enumerate(E.STEP_NAMES)}
PRE = BIT["ValidateWeights"] | BIT["ValidateReplicas"] | BIT["FillDefaults"]


def compare_masks(eng, opl, cfg, masks, osem):
    """The engine and the oracle call by call over the same masks: 'ok', 'error' (both
    failed alike at the same call) or 'dup-stop' (Go semantics: a remove left duplicated
    replicas and the mask skips ValidateReplicas -- the reference goes on over them, the
    engine stops with an explicit KB_ERR_UNSUPPORTED rather than guess)."""
    for i, m in enumerate(masks):
        r = O.step(opl, cfg, m, osem)
        try:
            g = eng.step(m)
        except E.EngineError as ex:
            if ex.code == -3 and "duplicated replicas" in str(ex):
                return "dup-stop"
            assert r["status"] < 0, (i, str(ex), r)
            if ": panic" not in r["err"]:
                assert str(ex) == r["err"], (i, str(ex), r["err"])
            return "error"
        assert r["status"] >= 0, (i, r["err"], g)
        if r["status"] == 0:
            assert g is None, (i, m, g)
            continue
        assert g is not None, (i, m, r)
        assert_same_plan([g], None, [r], None)
    return "ok"


def walk_table(eng, steps):
    """Balance() as the reference's loop over its steps table, one kb_engine_step per entry."""
    out = []
    for _ in range(steps):
        ch = None
        for k in range(9):
            ch = eng.step(1 << k)
            if ch is not None:
                break
        if ch is None:
            break
        out.append(ch)
    return out


# ----------------------------------------------------------- the steps table walk

CASES = []
for seed in range(24):
    r = random.Random(500 + seed)
    CASES.append(dict(seed=seed, P=r.choice([8, 20, 60, 150]), B=r.choice([3, 4, 6, 10, 25]),
                      weights=r.choice(["uniform", "int", "zipf"]), sets=r.choice(["none", "some", "all"]),
                      nrvar=r.random() < 0.5, ncons=r.random() < 0.3,
                      allow_leader=r.random() < 0.5, rebalance=r.random() < 0.25,
                      min_replicas=r.choice([1, 2, 2, 3]), min_unbalance=r.choice([0.0, 0.0, 1e-6]),
                      explicit=r.random() < 0.25, sem=r.choice(["applied", "go"])))


def case_input(case):
    rng = random.Random(9000 + case["seed"])
    pl = random_plist(rng, case["P"], case["B"], case["weights"], case["sets"], case["nrvar"], case["ncons"])
    cfg = default_cfg(allow_leader=case["allow_leader"], rebalance_leaders=case["rebalance"],
                      min_replicas=case["min_replicas"], min_unbalance=case["min_unbalance"])
    if case["explicit"]:
        cfg["brokers"] = list(range(1, case["B"] + 3))
    return pl, cfg


@pytest.mark.parametrize("case", CASES, ids=lambda c: "s%d" % c["seed"])
def test_steps_table_walk_matches_balance(case):
    """Balance() as a host loop over the table, one kb_engine_step per entry: the oracle's
    Balance() sequence (balancer.go:49-65), the same final state."""
    pl, cfg = case_input(case)
    sem = case["sem"]
    eng = E.Engine(pl, cfg, semantics=SEM[sem][0])
    try:
        got, gerr = walk_table(eng, 30), None
    except E.EngineError as ex:
        got, gerr = [], ex
    o = O.OraclePL(pl)
    want, werr = [], None
    for _ in range(30):
        r = O.balance(o, cfg, SEM[sem][1])
        if r["status"] == 0:
            break
        if r["status"] < 0:
            werr = r["err"]
            break
        want.append(r)
    if gerr is not None or werr is not None:
        # (the walk raises at the failing step: compare the prefix and the message)
        assert (gerr is None) == (werr is None), (gerr, werr)
        if ": panic" not in werr:
            assert str(gerr) == werr
        return
    assert_same_plan(got, None, want, None)
    assert eng.state() == o.state()
    eng.close()


# -------------------------------------------------------- single steps on their own

SINGLE = ["RemoveExtraReplicas", "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders",
          "MoveLeaders", "MoveNonLeaders"]


@pytest.mark.parametrize("sem", ["applied", "go"])
@pytest.mark.parametrize("name", SINGLE)
def test_single_step_alone_matches_oracle(name, sem):
    """One step function called repeatedly on its own (the rest of the table never runs):
    move() with disallowed and extra replicas still present, the first-index stages
    without move(), ReassignLeaders alone."""
    n = 0
    for seed in range(12):
        rng = random.Random(300 + seed)
        pl = random_plist(rng, rng.choice([20, 60, 120]), rng.choice([4, 6, 10]), rng.choice(["zipf", "int", "uniform"]),
                          rng.choice(["some", "all"]), True, rng.random() < 0.3)
        cfg = default_cfg(allow_leader=True, rebalance_leaders=True, min_unbalance=0.0,
                          min_replicas=rng.choice([1, 2]))
        eng = E.Engine(pl, cfg, semantics=SEM[sem][0])
        o = O.OraclePL(pl)
        r0 = O.step(o, cfg, PRE, SEM[sem][1])           # (the engine validated and filled at create)
        if r0["status"] != 0:
            continue
        masks = [BIT[name]] * 12
        if compare_masks(eng, o, cfg, masks, SEM[sem][1]) == "ok":
            assert eng.state() == o.state(), seed
        eng.close()
        n += 1
    assert n >= 8


@pytest.mark.parametrize("sem", ["applied", "go"])
def test_random_masks_match_oracle(sem):
    """Random subsets of the table per call (the no-change records reused across calls)."""
    names = E.STEP_NAMES
    for seed in range(16):
        rng = random.Random(4000 + seed)
        pl = random_plist(rng, rng.choice([30, 80]), rng.choice([5, 8]), rng.choice(["zipf", "uniform"]),
                          rng.choice(["none", "some"]), True, False)
        cfg = default_cfg(allow_leader=rng.random() < 0.7, rebalance_leaders=rng.random() < 0.3,
                          min_unbalance=0.0)
        masks = []
        for _ in range(40):
            k = rng.randint(1, 4)
            masks.append(sum(BIT[n] for n in rng.sample(names, k)))
        eng = E.Engine(pl, cfg, semantics=SEM[sem][0])
        o = O.OraclePL(pl)
        if O.step(o, cfg, PRE, SEM[sem][1])["status"] != 0:
            eng.close()
            continue
        if compare_masks(eng, o, cfg, masks, SEM[sem][1]) == "ok":
            assert eng.state() == o.state(), seed
            if sem == "applied":
                st = o.state()
                ws = [o.partition(i)["weight"] for i in range(o.n)]
                ncs = [o.partition(i)["num_consumers"] for i in range(o.n)]
                want_l = oracle_loads(st, ws, ncs)
                got_l = eng.loads()
                for b, v in want_l.items():
                    assert got_l[b] == v, (seed, b)
        eng.close()


def test_balancer_golden_cases_by_step():
    """The 16 TestBalancing cases (balancer_test.go:36-186) through the steps-table walk."""
    g = golden("balancer_cases.json")
    for c in g["cases"]:
        cfg = default_cfg(**g["configs"][c["cfg"]])
        pl = {"version": 1, "partitions": c["pl"]}
        eng = E.Engine(pl, cfg, semantics=E.KB_SEM_APPLIED)
        if "err" in c:
            with pytest.raises(E.EngineError) as ei:
                walk_table(eng, 1)
            r = O.balance(O.OraclePL(pl), cfg)
            assert str(ei.value) == r["err"], c["line"]
        elif c["ppl"] is None:
            assert walk_table(eng, 1) == [], c["line"]
        else:
            ch = walk_table(eng, 1)[0]
            exp = c["ppl"][0]
            got_p = pl["partitions"][ch["pidx"]]
            assert (got_p["topic"], got_p["partition"]) == (exp["topic"], exp["partition"]), c["line"]
            assert eng.replicas(ch["pidx"]) == exp["replicas"], c["line"]
        eng.close()


def test_validation_bits_and_pending_errors():
    """ValidateWeights / FillDefaults bits alone change nothing; a create-time validation
    error is returned by its own step and every later one, not by earlier ones."""
    pl = golden("test.json")
    eng = E.Engine(pl, default_cfg())
    assert eng.step(["ValidateWeights"]) is None
    assert eng.step(["FillDefaults"]) is None
    assert eng.step(["ValidateWeights", "ValidateReplicas", "FillDefaults"]) is None
    eng.close()
    bad = {"version": 1, "partitions": [dict(p) for p in pl["partitions"]]}
    bad["partitions"][1]["replicas"] = [1, 1]
    eng = E.Engine(bad, default_cfg())
    assert eng.step(["ValidateWeights"]) is None
    with pytest.raises(E.EngineError) as ei:
        eng.step(["ValidateReplicas"])
    r = O.balance(O.OraclePL(bad), default_cfg())
    assert str(ei.value) == r["err"]
    with pytest.raises(E.EngineError):
        eng.step(["MoveNonLeaders"])
    eng.close()


# ---------------------------------------------------------------------- at scale

@pytest.mark.parametrize("workload", ["c3", "c4"])
def test_table_walk_at_scale_matches_plan(workload):
    """c3 / c4 shapes (2 % scale): the host table walk (one kb_engine_step per entry, the
    scan of a no-change step reused by the next entry) equals kb_engine_plan's changes,
    bit for bit, and the same final loads."""
    cl, cfg, _ = synth.config(workload, scale=0.02)
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(40)
    assert err is None, err
    eng = E.Engine(cl, cfg)
    got = walk_table(eng, 40)
    assert got == want
    assert eng.loads() == ref.loads()
    ref.close()
    eng.close()


@pytest.mark.parametrize("shape", ["c3", "zipf4096"])
def test_table_walk_full_size_reuses_fused_records(shape):
    """The scan-reuse path (a masked step that changed nothing leaves its scan records to the
    next masked step, no second scan) on the production launches: c3 at full size (fused
    k_pair launches) and 1M partitions x 4096 brokers, Zipf (fused launches with eager
    refolds and fold checkpoints).  The host table walk equals kb_engine_plan change for
    change, with bit-identical loads after it."""
    if shape == "c3":
        cl, cfg, _ = synth.config("c3", scale=1.0)
        steps = 20
    else:
        cl = synth.make_cluster(1_000_000, 4096, 3, "zipf", seed=0x5EED5005)
        cfg = {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2, "min_unbalance": 0.0,
               "brokers": None}
        steps = 12
    ref = E.Engine(cl, cfg)
    want, err = ref.plan(steps)
    assert err is None, err
    assert ref.stats()["fused_pairs"] == 1
    eng = E.Engine(cl, cfg)
    got = walk_table(eng, steps)
    assert got == want
    assert eng.loads() == ref.loads()
    ref.close()
    eng.close()


def test_step_mask_names_combine_once():
    """A repeated step name sets its bit once; unknown names and masks outside the table are
    rejected before the C call."""
    pl = golden("test.json")
    eng = E.Engine(pl, default_cfg())
    a = eng.step(["MoveNonLeaders", "MoveNonLeaders"])
    eng2 = E.Engine(pl, default_cfg())
    b = eng2.step(["MoveNonLeaders"])
    assert a == b
    with pytest.raises(ValueError):
        eng.step(["MoveSideways"])
    with pytest.raises(ValueError):
        eng.step(1 << 9)
    eng.close()
    eng2.close()
