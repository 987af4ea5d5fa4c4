"""Diagnostic: one small plan (tests/golden/test.json, -allow-leader, 10 steps) on the
engine vs the oracle; prints the first divergence and the engine's plan counters."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kafkabalancer_amd import engine as E  # noqa: E402
from oracle import oracle as O  # noqa: E402

pl = json.load(open(os.path.join(ROOT, "tests", "golden", "test.json")))
cfg = dict(O.default_cfg(), allow_leader=True)
eng = E.Engine(pl, cfg)
ch, err = eng.plan(10)
o = O.OraclePL(pl)
want = []
for _ in range(10):
    r = O.balance(o, cfg, O.SEM_APPLIED)
    if r["status"] != 1:
        break
    want.append((r["step"], r["pidx"], r["from_"], r["to"], r["su"], r["cu"]))
got = [(c["step"], c["pidx"], c["from_"], c["to"], c["su"], c["cu"]) for c in ch]
st = eng.stats()
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("KB_")}, "match": [g[:4] == w[:4] for g, w in zip(got, want)],
                  "ngot": len(got), "nwant": len(want), "err": str(err) if err else None,
                  "launches": st["plan_launches"], "aborts": st["plan_aborts"], "got": got[:6], "want": want[:6]}))
