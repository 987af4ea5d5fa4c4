"""Shared test helpers: run the oracle and the engine side by side."""
import json
import math
import os

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def default_cfg(**kw):
    c = O.default_cfg()
    c.update(kw)
    return c


def oracle_plan(plist, cfg, steps, sem=O.SEM_APPLIED):
    """Balance() called `steps` times on the oracle; returns (changes, err, OraclePL)."""
    o = O.OraclePL(plist)
    changes = []
    for _ in range(steps):
        r = O.balance(o, cfg, sem)
        if r["status"] == 0:
            break
        if r["status"] < 0:
            return changes, r["err"], o
        changes.append(r)
    return changes, None, o


def key(ch):
    return (ch["step"], ch["pidx"], ch["kind"], ch["from_"], ch["to"], ch["slot"])


def rel_close(a, b, tol=1e-9):
    if a == b:
        return True
    if math.isnan(a) and math.isnan(b):
        return True
    return abs(a - b) <= tol * max(abs(a), abs(b), 1e-300)


def assert_same_plan(eng_changes, eng_err, orc_changes, orc_err):
    n = min(len(eng_changes), len(orc_changes))
    for i in range(n):
        e, o = eng_changes[i], orc_changes[i]
        assert key(e) == key(o), "step %d differs: engine %s oracle %s" % (i, key(e), key(o))
        if o["step"] in ("MoveLeaders", "MoveNonLeaders"):
            # 1e-9 relative to the unbalance scale of the step (the reference's own
            # fold noise at cu ~ 0 is ~1e-17 * su); bit-exact when the engine folded
            scale = max(abs(o["su"]), abs(o["cu"]), 1e-300)
            assert abs(e["su"] - o["su"]) <= 1e-9 * scale, (i, e["su"], o["su"])
            assert abs(e["cu"] - o["cu"]) <= 1e-9 * scale, (i, e["cu"], o["cu"])
            if e.get("exact"):
                # the engine folded in the reference's order: bit-exact
                assert e["cu"] == o["cu"], (i, e["cu"], o["cu"])
                assert e["su"] == o["su"], (i, e["su"], o["su"])
    assert len(eng_changes) == len(orc_changes), (len(eng_changes), len(orc_changes),
                                                  eng_err, orc_err)
    if orc_err is None:
        assert eng_err is None, str(eng_err)
    else:
        assert eng_err is not None, orc_err
        if ": panic" in orc_err:
            assert ": panic" in str(eng_err), (str(eng_err), orc_err)
        else:
            assert str(eng_err) == orc_err, (str(eng_err), orc_err)


def oracle_loads(state, weights, ncons):
    """getBrokerLoad (utils.go:92-105) of an explicit state, sequential in partition order."""
    loads = {}
    for reps, w, nc in zip(state, weights, ncons):
        for k, r in enumerate(reps):
            c = w * float(len(reps) + nc) if k == 0 else w
            loads[r] = loads.get(r, 0.0) + c
    return loads
