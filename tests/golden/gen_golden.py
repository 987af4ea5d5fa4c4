"""Generate tests/golden/plans_small.json from the CPU oracle (oracle/kb_oracle.c).

The reference is Go and cannot run here (no toolchain); these
plans are pinned by the oracle, which itself reproduces all 16 TestBalancing
cases of the reference (tests/test_oracle.py) and is cross-checked against an
independent Python restatement (oracle/pyref.py).

Run:  python tests/golden/gen_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402


def plan(name, plist, cfg, steps, sem):
    o = O.OraclePL(plist)
    changes, err = [], None
    s = O.SEM_GO if sem == "go" else O.SEM_APPLIED
    for _ in range(steps):
        r = O.balance(o, cfg, s)
        if r["status"] == 0:
            break
        if r["status"] < 0:
            err = r["err"]
            break
        changes.append([r["step"], r["pidx"], r["kind"], r["from_"], r["to"], r["slot"]])
    return {"name": name, "plist": plist, "cfg": cfg, "steps": steps, "sem": sem,
            "changes": changes, "err": err, "final": o.state()}


def main():
    from test_gpu_parity_data import random_plist  # noqa
    test_json = json.load(open(os.path.join(HERE, "test.json")))
    cases = []
    base = O.default_cfg()
    for sem in ("applied", "go"):
        cases.append(plan("c1-default-" + sem, test_json, dict(base), 20, sem))
        cases.append(plan("c1-leader-" + sem, test_json, dict(base, allow_leader=True), 12, sem))
        cases.append(plan("c1-rebalance-" + sem, test_json,
                          dict(base, rebalance_leaders=True, min_unbalance=0.0), 12, sem))
        cases.append(plan("c1-brokers6-" + sem, test_json, dict(base, brokers=[1, 2, 3, 4, 5, 6]), 20, sem))
    for seed in range(12):
        rng = random.Random(seed)
        pl = random_plist(rng, rng.choice([10, 30, 80]), rng.choice([3, 5, 9]),
                          rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                          rng.random() < 0.5, rng.random() < 0.3)
        cfg = dict(base, allow_leader=rng.random() < 0.5, min_unbalance=rng.choice([0.0, 0.01]),
                   min_replicas=rng.choice([1, 2, 3]))
        cases.append(plan("random-%d" % seed, pl, cfg, 25, rng.choice(["applied", "go"])))
    out = {"generator": "tests/golden/gen_golden.py (oracle/kb_oracle.c)", "cases": cases}
    with open(os.path.join(HERE, "plans_small.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
