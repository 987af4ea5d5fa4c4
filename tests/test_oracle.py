"""CPU tests: the oracle is pinned by the reference's own test vectors.

- the 16 TestBalancing cases (reference balancer_test.go:36-186), as data in
  tests/golden/balancer_cases.json
- the c1 plans predicted by SURVEY.md 8c
- cross-check of the C oracle against the independent Python restatement
  (oracle/pyref.py) on random tie-heavy multi-step plans
- Go encoding/json float formatting against Python's shortest repr
"""
import copy
import json
import os
import random
import struct

import pytest

from oracle import oracle as O
from oracle import pyref

from helpers import GOLDEN, default_cfg, golden
from test_gpu_parity_data import random_plist


def test_reference_balancer_cases():
    g = golden("balancer_cases.json")
    assert len(g["cases"]) == 16
    for c in g["cases"]:
        cfg = default_cfg(**g["configs"][c["cfg"]])
        r = O.balance(O.OraclePL({"version": 1, "partitions": c["pl"]}), cfg, O.SEM_GO)
        if "err" in c:
            assert r["status"] == -1 and c["err"] in r["err"], (c["line"], r)
        elif c["ppl"] is None:
            assert r["status"] == 0, (c["line"], r)
        else:
            e = c["ppl"][0]
            p = r["partition"]
            assert r["status"] == 1, c["line"]
            for k in ("topic", "partition", "replicas", "weight", "num_replicas", "brokers"):
                assert p[k] == e[k], (c["line"], k, p[k], e[k])
            assert p["num_consumers"] == e.get("num_consumers", 0)


def test_pyref_reference_cases():
    g = golden("balancer_cases.json")
    for c in g["cases"]:
        cfg = default_cfg(**g["configs"][c["cfg"]])
        pl = pyref.normalize({"partitions": c["pl"]})
        try:
            r = pyref.balance(pl, cfg)
        except pyref.StepError as ex:
            assert "err" in c and c["err"] in str(ex), (c["line"], ex)
            continue
        if c.get("ppl") is None:
            assert r is None and "err" not in c, c["line"]
        else:
            e = c["ppl"][0]
            assert pl[r[1]]["replicas"] == e["replicas"], c["line"]


def test_c1_predicted_plans():
    """SURVEY.md 8c predictions for test/test.json."""
    pl = golden("test.json")
    code, out, _ = O.run_plan(O.OraclePL(pl), O.default_cfg())
    assert code == 0
    assert out == (b'{"version":1,"partitions":[{"topic":"foo2","partition":1,"replicas":[4,2],'
                   b'"weight":1,"num_replicas":2,"brokers":[1,2,3,4]}]}\n')
    code, out, _ = O.run_plan(O.OraclePL(pl), O.default_cfg(), max_reassign=1000)
    assert code == 0 and out.count(b'"topic"') == 2
    # -allow-leader: a 2-cycle on foo2/0 from step 5 on, and the
    # default -complete-partition then never terminates
    cfg = dict(O.default_cfg(), allow_leader=True)
    o = O.OraclePL(pl)
    seq = [O.balance(o, cfg)["pidx"] for _ in range(9)]
    assert len(set(seq[:5])) == 5 and set(seq[5:]) == {3}
    code, _, _ = O.run_plan(O.OraclePL(pl), cfg, max_reassign=3, complete_partition=True)
    assert code == 0      # completion stops at the next (different) partition
    code, _, _ = O.run_plan(O.OraclePL(pl), cfg, max_reassign=6, complete_partition=True)
    assert code == 99     # the 6th move is foo2/0, which then flips forever


EMPTY_AFTER_PICK = {"version": 1, "partitions": [
    {"topic": "t", "partition": 0, "replicas": [1, 2], "weight": 5.0},
    {"topic": "t", "partition": 1, "replicas": [2, 3], "weight": 1.0},
    {"topic": "t", "partition": 2, "replicas": [], "weight": 1.0}]}


def test_distribute_leaders_empty_partition_after_pick_panics():
    """distributeLeaders builds pp over EVERY partition (steps.go:257-262) before it
    picks, so p.Replicas[0] panics on an empty list even when an eligible
    heavy-leader partition (P0) comes first."""
    cfg = default_cfg(rebalance_leaders=True, min_unbalance=0.0)
    for sem in (O.SEM_APPLIED, O.SEM_GO):
        r = O.balance(O.OraclePL(EMPTY_AFTER_PICK), cfg, sem)
        assert r["status"] == -1 and r["err"].startswith("ReassignLeaders: panic"), r
    with pytest.raises(pyref.StepError, match="panic"):
        pyref.balance(pyref.normalize(EMPTY_AFTER_PICK), cfg)
    # without -rebalance-leader the step is skipped and move() only reads slots of
    # eligible partitions (P2 has NumReplicas 0 < MinReplicas): no panic
    r = O.balance(O.OraclePL(EMPTY_AFTER_PICK), default_cfg(min_unbalance=0.0), O.SEM_APPLIED)
    assert r["status"] >= 0, r


def _pyref_plan(plist, cfg, steps):
    pl = pyref.normalize(plist)
    out = []
    try:
        for _ in range(steps):
            r = pyref.balance(pl, cfg)
            if r is None:
                break
            out.append(r)
    except pyref.StepError as ex:
        return out, str(ex), pl
    return out, None, pl


@pytest.mark.parametrize("seed", range(60))
def test_oracle_vs_pyref(seed):
    rng = random.Random(seed)
    pl = random_plist(rng, rng.choice([4, 12, 40]), rng.choice([2, 3, 5, 8]),
                      rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                      rng.random() < 0.4, rng.random() < 0.3)
    cfg = default_cfg(allow_leader=rng.random() < 0.5, rebalance_leaders=rng.random() < 0.3,
                      min_replicas=rng.choice([1, 2, 3]), min_unbalance=rng.choice([0.0, 0.01]))
    if rng.random() < 0.3:
        cfg["brokers"] = list(range(1, 10))
    steps = 15
    pch, perr, ppl = _pyref_plan(copy.deepcopy(pl), cfg, steps)
    o = O.OraclePL(pl)
    och = []
    oerr = None
    for _ in range(steps):
        r = O.balance(o, cfg, O.SEM_APPLIED)
        if r["status"] == 0:
            break
        if r["status"] < 0:
            oerr = r["err"]
            break
        och.append((r["step"], r["pidx"], r["kind"] if r["kind"] != "swap" else "swap", r["from_"], r["to"]))
    assert [(a[0], a[1], a[3], a[4]) for a in pch] == [(a[0], a[1], a[3], a[4]) for a in och]
    if perr is None:
        assert oerr is None
        assert [p["replicas"] for p in ppl] == o.state()
    else:
        assert oerr is not None
        if "panic" not in perr:
            assert perr == oerr


@pytest.mark.parametrize("seed", range(12))
def test_threaded_oracle_matches_sequential(seed):
    """or_set_threads(T): chunked move() / Disallowed search, merged in order --
    the identical plan, unbalance bits and errors as T = 1."""
    rng = random.Random(500 + seed)
    pl = random_plist(rng, rng.choice([40, 90, 200]), rng.choice([3, 6, 12]),
                      rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                      rng.random() < 0.4, rng.random() < 0.3)
    cfg = default_cfg(allow_leader=rng.random() < 0.5, rebalance_leaders=rng.random() < 0.2,
                      min_replicas=rng.choice([1, 2, 3]), min_unbalance=rng.choice([0.0, 0.01]))

    def run(threads):
        O.set_threads(threads)
        try:
            o = O.OraclePL(pl)
            out = []
            for _ in range(20):
                r = O.balance(o, cfg, O.SEM_APPLIED)
                out.append((r["status"], r["step"], r.get("pidx"), r.get("from_"), r.get("to"),
                            r.get("su"), r.get("cu"), r["err"]))
                if r["status"] != 1:
                    break
            return out, o.state()
        finally:
            O.set_threads(1)

    assert run(1) == run(5)


def test_golden_plans_reproduce():
    """The committed oracle plans (gen_golden.py) still come out of the oracle."""
    g = golden("plans_small.json")
    assert len(g["cases"]) >= 20
    for case in g["cases"]:
        o = O.OraclePL(case["plist"])
        sem = O.SEM_GO if case["sem"] == "go" else O.SEM_APPLIED
        got, err = [], None
        for _ in range(case["steps"]):
            r = O.balance(o, case["cfg"], sem)
            if r["status"] == 0:
                break
            if r["status"] < 0:
                err = r["err"]
                break
            got.append([r["step"], r["pidx"], r["kind"], r["from_"], r["to"], r["slot"]])
        assert got == case["changes"], case["name"]
        assert err == case["err"], case["name"]
        assert o.state() == case["final"], case["name"]


def go_float(x):
    """Go encoding/json float64 text, from Python's shortest round-trip digits."""
    import decimal
    if x == 0:
        return "0"
    sign = "-" if x < 0 else ""
    a = abs(x)
    t = decimal.Decimal(repr(a)).normalize().as_tuple()
    digits = "".join(map(str, t.digits))
    point = len(digits) + t.exponent          # value = 0.digits * 10^point
    if a < 1e-6 or a >= 1e21:
        e = point - 1
        mant = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        return sign + mant + (("e-%d" % -e) if e < 0 else ("e+%02d" % e))
    if point <= 0:
        return sign + "0." + "0" * (-point) + digits
    if point >= len(digits):
        return sign + digits + "0" * (point - len(digits))
    return sign + digits[:point] + "." + digits[point:]


def test_go_float_format():
    rng = random.Random(7)
    vals = [1.0, 0.5, 0.1, 1e-7, 2.5e-7, 1e-6, 123456.789, 1e20, 1e21, 3e22, 1 / 3, 2.0 ** -30,
            0.000123, 1e300, 5e-324, 7.0, 100.0]
    vals += [rng.uniform(1, 1e6) ** -1.1 for _ in range(300)]
    vals += [rng.uniform(0, 1e7) for _ in range(200)]
    for v in vals:
        assert O.format_float(v) == go_float(v), v
        assert float(O.format_float(v)) == v


def test_json_writer_matches_go_layout():
    pl = {"version": 1, "partitions": [
        {"topic": "a<b>&c", "partition": 3, "replicas": [2, 1], "weight": 2.5e-7, "num_consumers": 2},
        {"topic": "x", "partition": 0, "replicas": [1, 2]}]}
    code, out, _ = O.run_plan(O.OraclePL(pl), O.default_cfg(), full_output=True, max_reassign=0)
    assert code == 0
    want = ('{"version":1,"partitions":[{"topic":"a\\u003cb\\u003e\\u0026c","partition":3,'
            '"replicas":[2,1],"weight":2.5e-7,"num_consumers":2},'
            '{"topic":"x","partition":0,"replicas":[1,2]}]}\n').encode()
    assert out == want
    json.loads(out)


@pytest.mark.parametrize("seed", range(16))
def test_windowed_oracle_matches_literal(seed):
    """or_set_window(1) (golden generation: O(1) scores, exact folds only inside the window
    that holds the reference's choice) -- the identical plan, su / cu bits and errors as the
    literal move() loop, uniform exact-tie weights included."""
    rng = random.Random(900 + seed)
    pl = random_plist(rng, rng.choice([40, 90, 200]), rng.choice([3, 6, 12, 30]),
                      rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                      rng.random() < 0.4, rng.random() < 0.3)
    cfg = default_cfg(allow_leader=rng.random() < 0.5, rebalance_leaders=rng.random() < 0.2,
                      min_replicas=rng.choice([1, 2, 3]), min_unbalance=rng.choice([0.0, 0.01]))
    if rng.random() < 0.3:
        cfg["brokers"] = list(range(1, 40))

    def run(window, threads):
        O.set_threads(threads)
        O.set_window(window)
        try:
            o = O.OraclePL(pl)
            out = []
            for _ in range(25):
                r = O.balance(o, cfg, O.SEM_APPLIED)
                out.append((r["status"], r["step"], r.get("pidx"), r.get("from_"), r.get("to"),
                            r.get("su"), r.get("cu"), r["err"]))
                if r["status"] != 1:
                    break
            return out, o.state()
        finally:
            O.set_threads(1)
            O.set_window(0)

    assert run(0, 1) == run(1, 3)


# the early-stop target walk of the windowed search runs only with n >= 64 brokers
# (kb_oracle.c move_window); these plans exercise it against the literal loop: 64-200 brokers,
# every weight mode, with and without allowed lists, leader moves on and off
WALK_CASES = [(b, w, s, al) for b in (64, 97, 150, 200) for w in ("uniform", "int", "zipf")
              for s, al in (("none", False), ("all", True), ("some", False), ("all", False))]


@pytest.mark.parametrize("B,weights,sets,allow_leader", WALK_CASES)
def test_windowed_oracle_walk_matches_literal(B, weights, sets, allow_leader):
    """or_set_window(1) with the early-stop walk (n >= 64) equals the literal move() loop on
    the whole plan: every change, su / cu bit and the final state; the walk's stop branch
    is taken (its counter), so the n >= 64 path is what was compared."""
    rng = random.Random(hash((B, weights, sets, allow_leader)) & 0xFFFFFFFF)
    pl = random_plist(rng, rng.choice([300, 600]), B, weights, sets, False, rng.random() < 0.3)
    for p in pl["partitions"]:
        # (allowed lists that hold the partition's replicas: the plan reaches move() at once
        # instead of spending its steps in MoveDisallowedReplicas)
        if "brokers" in p:
            p["brokers"] = sorted(set(p["brokers"]) | set(p["replicas"]))
    cfg = default_cfg(allow_leader=allow_leader, min_unbalance=0.0)

    def run(window, threads):
        O.set_threads(threads)
        O.set_window(window)
        try:
            o = O.OraclePL(pl)
            out = []
            for _ in range(12):
                r = O.balance(o, cfg, O.SEM_APPLIED)
                out.append((r["status"], r["step"], r.get("pidx"), r.get("kind"), r.get("from_"), r.get("to"),
                            r.get("slot"), r.get("su"), r.get("cu"), r["err"]))
                if r["status"] != 1:
                    break
            return out, o.state()
        finally:
            O.set_threads(1)
            O.set_window(0)

    want = run(0, 1)
    O.walk_stops(reset=True)
    got = run(1, 3)
    stops = O.walk_stops(reset=True)
    assert got == want
    assert stops > 0, "the early-stop walk never ran"


@pytest.mark.parametrize("name", ["b4096_zipf", "b4096_uniform", "c3s_nonleader", "c3s_leader", "b6000_zipf"])
def test_windowed_oracle_reproduces_scale_goldens(name):
    """The windowed search regenerates the committed large goldens the literal loop made
    (4096 brokers; 20k partitions x 1000 brokers with 256 allowed sets, leader and
    non-leader moves): every change and every su / cu bit."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_scale", os.path.join(GOLDEN, "gen_scale.py"))
    gs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gs)
    g = golden("scale_%s.json" % name)
    params, _, steps = gs.CASES[name]
    cl = gs.build(params)
    assert gs.input_hash(cl) == g["input_sha256"]
    cfg = gs.case_cfg(name)
    O.set_threads(min(8, os.cpu_count() or 1))
    O.set_window(1)
    O.walk_stops(reset=True)
    # (b4096_uniform: the exact-tie worst case, and b6000_zipf: past the LDS broker tables;
    # their first 12 steps)
    nmax = 12 if name in ("b4096_uniform", "b6000_zipf") else 60
    try:
        o = gs.oracle_pl(cl)
        for k, want in enumerate(g["changes"][:nmax]):
            r = O.balance(o, cfg, O.SEM_APPLIED)
            assert r["status"] == 1, (k, r["err"])
            assert [r["step"], r["pidx"], r["kind"], r["from_"], r["to"], r["slot"]] == want, k
            assert r["su"] == g["su"][k] and r["cu"] == g["cu"][k], k
        # (n >= 64 brokers everywhere here: the early-stop walk ran)
        assert O.walk_stops(reset=True) > 0
    finally:
        O.set_threads(1)
        O.set_window(0)
