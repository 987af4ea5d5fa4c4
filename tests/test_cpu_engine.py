"""The OpenMP CPU engine (tools/cpu_engine, the optimised CPU baseline of bench.py)
computes the reference's plans: identical change sequences and su/cu bits against the
oracle (steps.go:145-232) on seeded clusters in every weight mode, with and without
allowed-broker sets and -allow-leader."""
import os
import sys

import pytest

from oracle import oracle as O
from kafkabalancer_amd import synth

from helpers import default_cfg

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "cpu_engine"))
import cpu_engine  # noqa: E402

CASES = [(P, B, wts, sets, al, thr) for P, B in ((60, 8), (400, 20), (2000, 60))
         for wts in ("uniform", "int", "zipf") for sets in (0, 1) for al in (False, True) for thr in (1, 4)][::3]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "P%d-B%d-%s-s%d-l%d-t%d" % c)
def test_cpu_engine_matches_oracle(case):
    P, B, wts, sets, al, thr = case
    kw = dict(nsets=6, set_size=max(4, B // 2)) if sets else {}
    cl = synth.make_cluster(P, B, 3, wts, seed=P * 7 + B, with_names=True, **kw)
    cfg = default_cfg(allow_leader=al, min_unbalance=0.0)
    ce = cpu_engine.CpuEngine(cl, cfg, threads=thr)
    o = O.OraclePL(synth.to_plist(cl))
    for k in range(15):
        r = O.balance(o, cfg, O.SEM_APPLIED)
        c = ce.step()
        if r["status"] != 1:
            assert c is None, (k, c)
            break
        assert c is not None, (k, r)
        assert (c["step"], c["pidx"], c["from_"], c["to"], c["slot"]) == (r["step"], r["pidx"], r["from_"], r["to"], r["slot"]), k
        assert (c["su"], c["cu"]) == (r["su"], r["cu"]), k
    ce.close()


@pytest.mark.parametrize("thr", [1, 4])
def test_cpu_engine_first_index_stages_match_oracle(thr):
    """c4's shape (broker add / decommission, replica-count changes): RemoveExtraReplicas,
    AddMissingReplicas and MoveDisallowedReplicas (steps.go:70-143) before move(), against
    the oracle step for step."""
    import numpy as np
    P, B = 3000, 80
    rng = np.random.default_rng(11)
    nr = np.zeros(P, np.int64)
    pick = rng.choice(P, size=60, replace=False)
    nr[pick[:30]] = 2
    nr[pick[30:]] = 4
    cl = synth.make_cluster(P, B, 3, "zipf", seed=0x5EED4404, with_names=True, num_replicas=nr)
    cfg = default_cfg(min_unbalance=0.0)
    cfg["brokers"] = [b for b in range(1, 91) if not 79 <= b <= 80]
    ce = cpu_engine.CpuEngine(cl, cfg, threads=thr)
    o = O.OraclePL(synth.to_plist(cl))
    seen = set()
    for k in range(420):
        r = O.balance(o, cfg, O.SEM_APPLIED)
        c = ce.step()
        if r["status"] != 1:
            assert c is None, (k, c)
            break
        assert c is not None, (k, r)
        seen.add(r["step"])
        assert (c["step"], c["pidx"], c["from_"], c["to"], c["slot"]) == (r["step"], r["pidx"], r["from_"], r["to"], r["slot"]), k
        if r["step"] in ("MoveLeaders", "MoveNonLeaders"):
            assert (c["su"], c["cu"]) == (r["su"], r["cu"]), k
    assert {"RemoveExtraReplicas", "AddMissingReplicas", "MoveDisallowedReplicas", "MoveNonLeaders"} <= seen, seen
    ce.close()
