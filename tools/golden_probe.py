"""Diagnostic: replay one tests/golden/scale_*.json plan on the engine; print where it
diverges from the oracle's and the engine's counters."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_scale  # noqa: E402
from kafkabalancer_amd import engine as E  # noqa: E402

name = sys.argv[1]
g = json.load(open(os.path.join(ROOT, "tests", "golden", "scale_%s.json" % name)))
cl = gen_scale.build(g["params"])
eng = E.Engine(cl, dict(g["cfg"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else g["steps"]
changes, err = eng.plan(steps)
got = [[c["step"], c["pidx"], c["kind"], c["from_"], c["to"], c["slot"]] for c in changes]
div = next((i for i, (a, b) in enumerate(zip(got, g["changes"])) if a != b), None)
st = eng.stats()
print(json.dumps({"case": name, "env": {k: v for k, v in os.environ.items() if k.startswith("KB_")},
                  "ngot": len(got), "nwant": min(len(g["changes"]), steps), "diverge": div,
                  "at": [got[div], g["changes"][div]] if div is not None else None,
                  "err": str(err) if err else None,
                  "stats": {k: st[k] for k in ("steps", "refreshes", "exact_halts", "retries")}}))
