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
