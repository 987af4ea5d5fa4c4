"""Independent pure-Python restatement of the reference balancer.

TEST INFRASTRUCTURE ONLY (small cases).  Written separately from kb_oracle.c
so the two restatements cross-check each other (tests/test_oracle.py).
Python floats are IEEE binary64 with no FMA, like Go on amd64.

Follows steps.go:7-307, utils.go:19-202, balancer.go:34-65.  State is kept
"applied" (a returned change is written back into the list), which equals the
reference's aliasing behaviour for every replace/swap move (utils.go:186-190).
"""

STEPS = ["ValidateWeights", "ValidateReplicas", "FillDefaults", "RemoveExtraReplicas",
         "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders", "MoveLeaders",
         "MoveNonLeaders"]


class StepError(Exception):
    pass


def pstr(p):
    return "Partition(%s,%d,[%s])" % (p["topic"], p["partition"],
                                       " ".join(str(r) for r in p["replicas"] or []))


def broker_load(pl):                       # utils.go:92-105
    loads = {}
    for p in pl:
        reps = p["replicas"] or []
        for i, r in enumerate(reps):
            c = p["weight"] * float(len(reps) + p["num_consumers"]) if i == 0 else p["weight"]
            loads[r] = loads.get(r, 0.0) + c
    return loads


def get_bl(loads):                         # utils.go:107-117
    return sorted(([b, l] for b, l in loads.items()), key=lambda x: (x[1], x[0]))


def unbalance(bl):                         # utils.go:119-147
    s = 0.0
    for _, l in bl:
        s += l
    avg = s / float(len(bl))
    u = 0.0
    for _, l in bl:
        r = l / avg - 1.0
        u += r * r if r > 0 else r * r / 2
    return u


def _replace(p, orig, repl):               # utils.go:166-197 (applied)
    reps = p["replicas"]
    for idx, b in enumerate(reps):
        if b != orig:
            continue
        if repl == -1:
            del reps[idx]
            return ("remove", idx)
        if repl in reps:
            e = reps.index(repl)
            reps[idx], reps[e] = repl, reps[idx]
            return ("swap", idx)
        reps[idx] = repl
        return ("replace", idx)
    raise StepError("panic")


def balance(pl, cfg):
    """One Balance() call; returns None (no change) or (step, pidx, kind, from, to); raises StepError."""
    if not pl:
        raise StepError("panic")
    # ValidateWeights
    has = pl[0]["weight"] != 0
    for p in pl:
        if has and p["weight"] == 0:
            raise StepError("ValidateWeights: partition %s has no weight" % pstr(p))
        if not has and p["weight"] != 0:
            raise StepError("ValidateWeights: partition %s has no weight" % pstr(pl[0]))
        if p["weight"] < 0:
            raise StepError("ValidateWeights: partition %s has negative weight" % pstr(p))
    for p in pl:
        reps = p["replicas"] or []
        if len(set(reps)) != len(reps):
            raise StepError("ValidateReplicas: partition %s has duplicated replicas" % pstr(p))
    # FillDefaults
    if pl[0]["weight"] == 0:
        for p in pl:
            p["weight"] = 1.0
    brokers = cfg["brokers"]
    if brokers is None:
        s = sorted({r for p in pl for r in (p["replicas"] or [])})
        brokers = s if s else None
    for p in pl:
        if p["brokers"] is None:
            p["brokers"] = brokers
    for p in pl:
        if p["num_replicas"] == 0:
            p["num_replicas"] = len(p["replicas"] or [])
    loads = broker_load(pl)
    # RemoveExtraReplicas
    for i, p in enumerate(pl):
        if p["num_replicas"] >= len(p["replicas"]):
            continue
        for b in sorted(p["brokers"] or [], key=lambda b: (loads.get(b, 0.0), b)):
            if b in p["replicas"]:
                _replace(p, b, -1)
                return ("RemoveExtraReplicas", i, "remove", b, -1)
        raise StepError("RemoveExtraReplicas: partition %s unable to pick replica to remove" % pstr(p))
    # AddMissingReplicas
    for i, p in enumerate(pl):
        if p["num_replicas"] <= len(p["replicas"]):
            continue
        for b in reversed(sorted(p["brokers"] or [], key=lambda b: (loads.get(b, 0.0), b))):
            if b not in p["replicas"]:
                p["replicas"].append(b)
                return ("AddMissingReplicas", i, "add", -1, b)
        raise StepError("AddMissingReplicas: partition %s unable to pick replica to add" % pstr(p))
    # MoveDisallowedReplicas
    bl = get_bl(loads)
    for i, p in enumerate(pl):
        allowed = set(p["brokers"] or [])
        A = [b for b, _ in bl if b in allowed]
        for r in list(p["replicas"]):
            if r in A:
                continue
            for b in reversed(A):
                if b in p["replicas"]:
                    continue
                _replace(p, r, b)
                return ("MoveDisallowedReplicas", i, "replace", r, b)
            raise StepError("MoveDisallowedReplicas: partition %s unable to pick replica to "
                            "replace broker %d" % (pstr(p), r))
    full = dict(loads)
    for b in cfg["brokers"] or []:
        full.setdefault(b, 0.0)
    # ReassignLeaders / distributeLeaders (steps.go:234-282)
    if cfg["rebalance_leaders"]:
        bl = get_bl(full)
        su = unbalance(bl)
        if not su < cfg["min_unbalance"]:
            heavy = bl[-1][0]
            # pp is built over every partition first (steps.go:257-262)
            if any(not p["replicas"] for p in pl):
                raise StepError("ReassignLeaders: panic")
            for i, p in enumerate(pl):
                if p["replicas"][0] != heavy or p["num_replicas"] < cfg["min_replicas"]:
                    continue
                r0 = p["replicas"][0]
                kind, _ = _replace(p, r0, bl[0][0])
                return ("ReassignLeaders", i, kind, r0, bl[0][0])
    for leaders in ([True] if cfg["allow_leader"] else []) + [False]:
        bl = get_bl(full)
        su = unbalance(bl)
        cu, best = su, None
        for i, p in enumerate(pl):
            if p["num_replicas"] < cfg["min_replicas"]:
                continue
            slots = p["replicas"][0:1] if leaders else p["replicas"][1:]
            allowed = set(p["brokers"] or [])
            for r in slots:
                ridx = [k for k, x in enumerate(bl) if x[0] == r][0]
                rload = bl[ridx][1]
                bl[ridx][1] -= p["weight"]
                for k, (b, l) in enumerate(bl):
                    if b not in allowed or b in p["replicas"]:
                        continue
                    bl[k][1] = l + p["weight"]
                    u = unbalance(bl)
                    if u < cu:
                        cu, best = u, (i, r, b)
                    bl[k][1] = l
                bl[ridx][1] = rload
        if cu < su - cfg["min_unbalance"]:
            i, r, b = best
            _replace(pl[i], r, b)
            return ("MoveLeaders" if leaders else "MoveNonLeaders", i, "replace", r, b)
    return None


def normalize(plist):
    """dict partitions -> mutable state with defaults for missing fields."""
    out = []
    for p in plist["partitions"]:
        out.append({"topic": p["topic"], "partition": p["partition"],
                    "replicas": list(p["replicas"]) if p.get("replicas") is not None else None,
                    "weight": float(p.get("weight", 0) or 0),
                    "num_replicas": int(p.get("num_replicas", 0) or 0),
                    "brokers": list(p["brokers"]) if p.get("brokers") is not None else None,
                    "num_consumers": int(p.get("num_consumers", 0) or 0)})
    return out
