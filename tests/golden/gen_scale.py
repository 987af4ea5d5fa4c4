"""Generate the large-scale golden plans tests/golden/scale_<name>.json from the CPU
oracle (oracle/kb_oracle.c, threaded move(): identical results for any thread count,
tests/test_oracle.py::test_threaded_oracle_matches_sequential).

These pin the engine's parity far beyond what the oracle can replay inside a test:
c3-shaped (1000 brokers, 256 allowed sets of 64, Zipf weights, -allow-leader and
without), a 4096-broker auto-list case in both weight modes (Zipf and the uniform
exact-tie worst case) and a c4-shaped broker add/remove case that runs through
RemoveExtraReplicas, AddMissingReplicas and MoveDisallowedReplicas into move().

Each fixture stores the synth parameters, a SHA-256 of the generated input arrays
(the GPU test regenerates the input and checks it first), the change list
[step, pidx, kind, from, to, slot] and su / cu of every step as exact floats.

Full-size cases (`c3_full`, `c4_full`) regenerate BASELINE.json's headline configs
themselves (kafkabalancer_amd/synth.config: c3 = 1M partitions x 1000 brokers, 256
allowed sets of 64, Zipf weights, -allow-leader; c4 = 1M partitions, 1000 -> 1150
allowed brokers with 50 decommissioned, 300 removes + 300 adds) and load them into the
oracle as arrays (OraclePL.from_soa), not through the dict form.  `rl20k` pins
distributeLeaders (steps.go:234-282, -rebalance-leader) at 20k partitions.

Run:  python tests/golden/gen_scale.py [case ...]   (all cases: ~30 min on 8 cores)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

from kafkabalancer_amd import synth  # noqa: E402


def c4_cfg():
    return dict(O.default_cfg(), min_unbalance=0.0,
                brokers=[b for b in range(1, 241) if not 196 <= b <= 200])


def c4_nr(P, seed):
    rng = np.random.default_rng(seed)
    nr = np.zeros(P, np.int64)
    pick = rng.choice(P, size=60, replace=False)
    nr[pick[:30]] = 2
    nr[pick[30:]] = 4
    return nr


# name -> (make_cluster kwargs, cfg, steps)
CASES = {
    "c3s_leader": (dict(P=20000, B=1000, rf=3, weights="zipf", nsets=256, set_size=64, seed=0x5EED1003),
                   dict(O.default_cfg(), allow_leader=True, min_unbalance=0.0), 200),
    "c3s_nonleader": (dict(P=20000, B=1000, rf=3, weights="zipf", nsets=256, set_size=64, seed=0x5EED2003),
                      dict(O.default_cfg(), min_unbalance=0.0), 200),
    "b4096_zipf": (dict(P=3000, B=4096, rf=3, weights="zipf", seed=0x5EED1005),
                   dict(O.default_cfg(), min_unbalance=0.0), 12),
    "b4096_uniform": (dict(P=3000, B=4096, rf=3, weights="uniform", seed=0x5EED2005),
                      dict(O.default_cfg(), min_unbalance=0.0), 12),
    "c4s": (dict(P=20000, B=200, rf=3, weights="zipf", seed=0x5EED1004, nr_seed=0x5EED1104),
            c4_cfg(), 1700),
    # BASELINE.json configs[2] at full size: the first 20 steps of the bench workload
    "c3_full": (dict(config="c3", scale=1.0), None, 20),
    # BASELINE.json configs[3] at full size: the whole 1000-step plan (Remove, Add,
    # Disallowed stages, steps.go:70-143)
    "c4_full": (dict(config="c4", scale=1.0), None, 1000),
    # -rebalance-leader (distributeLeaders, steps.go:234-282) with -allow-leader, 20k
    # partitions, c3-shaped sets
    "rl20k": (dict(P=20000, B=1000, rf=3, weights="zipf", nsets=256, set_size=64, seed=0x5EED3003),
              dict(O.default_cfg(), allow_leader=True, rebalance_leaders=True, min_unbalance=0.0), 200),
    # BASELINE.json configs[2]'s cluster without -allow-leader: MoveNonLeaders at 1M x 1000
    # with 256 allowed sets of 64 (the headline config's leader 2-cycle never reaches it)
    "c3nl_full": (dict(config="c3", scale=1.0), dict(O.default_cfg(), min_unbalance=0.0), 20),
    # c5's broker width (4096, auto lists, Zipf) at 50k partitions
    "b4096_50k": (dict(P=50000, B=4096, rf=3, weights="zipf", seed=0x5EED3005),
                  dict(O.default_cfg(), min_unbalance=0.0), 40),
    # BASELINE.json configs[4] at full size: 10M partitions x 4096 brokers, the first steps
    "c5_full": (dict(config="c5", scale=1.0), None, 12),
    # past the 4096 brokers the kernels keep in LDS (broker tables in memory): auto lists
    # with Zipf weights (eager refolds, exact folds), allowed sets with -allow-leader, the
    # integral mode at the engine's 16384-broker limit, and the uniform exact-tie case
    # (b8000_sets without -allow-leader: with it, the leader 2-cycle of SURVEY 3.4 repeats)
    "b6000_zipf": (dict(P=30000, B=6000, rf=3, weights="zipf", seed=0x5EED6000),
                   dict(O.default_cfg(), min_unbalance=0.0), 40),
    "b8000_sets": (dict(P=30000, B=8000, rf=3, weights="zipf", nsets=200, set_size=64, seed=0x5EED8000),
                   dict(O.default_cfg(), min_unbalance=0.0), 60),
    "b16384_int": (dict(P=60000, B=16384, rf=3, weights="int", seed=0x5EED4000),
                   dict(O.default_cfg(), min_unbalance=0.0), 30),
    "b12000_uniform": (dict(P=40000, B=12000, rf=3, weights="uniform", seed=0x5EEDC000),
                       dict(O.default_cfg(), min_unbalance=0.0), 12),
    # the benchmarked plans end to end: BASELINE.json configs[2]'s whole 1000-move plan (the
    # headline, -allow-leader), the same cluster's 1000 MoveNonLeaders steps without
    # -allow-leader, and configs[4] (c5) over the 200 steps bench.py times there; their
    # first 20 / 20 / 12 steps are c3_full, c3nl_full and c5_full (tests/test_golden_scale.py)
    "c3_full1000": (dict(config="c3", scale=1.0), None, 1000),
    "c3nl_1000": (dict(config="c3", scale=1.0), dict(O.default_cfg(), min_unbalance=0.0), 1000),
    "c5_200": (dict(config="c5", scale=1.0), None, 200),
}

# cases generated with the oracle's windowed exact move() (or_set_window: the literal
# loop's result, tests/test_oracle.py::test_windowed_oracle_*; the literal loop would take
# hours to days per step at these sizes)
WINDOWED = {"c3nl_full", "b4096_50k", "c5_full", "b6000_zipf", "b8000_sets", "b16384_int", "b12000_uniform",
            "c3_full1000", "c3nl_1000", "c5_200"}


def build(params):
    if "config" in params:
        return synth.config(params["config"], scale=params["scale"])[0]
    kw = dict(params)
    nr_seed = kw.pop("nr_seed", None)
    P = kw.pop("P")
    B = kw.pop("B")
    nr = c4_nr(P, nr_seed) if nr_seed is not None else None
    return synth.make_cluster(P, B, kw.pop("rf"), kw.pop("weights"), nsets=kw.pop("nsets", 0),
                              set_size=kw.pop("set_size", 0), seed=kw.pop("seed"), with_names=True,
                              num_replicas=nr)


def input_hash(cl):
    h = hashlib.sha256()
    for a in (cl.replica_ids, cl.replica_off, cl.weight, cl.num_replicas, cl.set_ids, cl.set_off, cl.set_idx):
        if a is not None:
            h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def case_cfg(name):
    params, cfg, _ = CASES[name]
    if cfg is None:
        cfg = synth.config(params["config"], scale=params["scale"])[1]
    return cfg


def oracle_pl(cl):
    """Large clusters go into the oracle as arrays (the dict form of 1M partitions with
    64-broker lists would need tens of GB of Python objects).  Weight / NumReplicas stay
    raw: the oracle's FillDefaults (steps.go:39-66) fills them like the reference."""
    if cl.n <= 100000:
        return O.OraclePL(synth.to_plist(cl))
    P = cl.n
    return O.OraclePL.from_soa(b"t", np.zeros(P + 1, np.int64), np.arange(P, dtype=np.int64) % 100,
                               cl.replica_ids, cl.replica_off, cl.weight, cl.num_replicas,
                               cl.set_ids, cl.set_off, cl.set_idx, cl.num_consumers)


def generate(name, threads):
    params, _, steps = CASES[name]
    cfg = case_cfg(name)
    cl = build(params)
    O.set_threads(threads)
    O.set_window(name in WINDOWED)
    o = oracle_pl(cl)
    changes, su, cu, err = [], [], [], None
    t0 = time.time()
    for k in range(steps):
        r = O.balance(o, cfg, O.SEM_APPLIED)
        if r["status"] == 0:
            break
        if r["status"] < 0:
            err = r["err"]
            break
        changes.append([r["step"], r["pidx"], r["kind"], r["from_"], r["to"], r["slot"]])
        su.append(r["su"])
        cu.append(r["cu"])
        if k % 20 == 0:
            print(name, k, r["step"], "%.0fs" % (time.time() - t0), flush=True)
    # final replicas of every partition some change touched
    touched = sorted({c[1] for c in changes})
    doc = {"name": name, "generator": "tests/golden/gen_scale.py (oracle/kb_oracle.c, %d threads%s)"
                                      % (threads, ", windowed exact move()" if name in WINDOWED else ""),
           "params": params, "cfg": cfg, "steps": steps, "input_sha256": input_hash(cl),
           "changes": changes, "su": su, "cu": cu, "err": err,
           "final": {str(i): o.replicas(i) for i in touched}}
    with open(os.path.join(HERE, "scale_%s.json" % name), "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print("wrote", name, len(changes), "changes in %.0fs" % (time.time() - t0), flush=True)


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)
    for n in names:
        generate(n, os.cpu_count() or 1)
