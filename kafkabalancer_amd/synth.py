"""Synthetic cluster generators for the BASELINE.json configurations.

SURVEY.md 8d: broker ids 1..B, topic "t%05d" with 100 partitions each, weights
absent (-> 1.0) or Zipf-like w = r^-1.1 with r uniform in [1, 1e6], allowed
sets drawn per partition.  Deterministic for a seed.  SURVEY 8d named splitmix64;
the generator is numpy's PCG64 instead (vectorised draws for 10M partitions): no
reference-run numbers exist for these inputs, so the stream only has to be fixed and
reproducible -- the golden fixtures regenerate from it bit-identically
(tests/test_golden_scale.py).
Returns (ClusterSoA, cfg dict, description).
"""
import numpy as np

from .engine import ClusterSoA


def _distinct(rng, n_choices, count, rf):
    """count x rf distinct draws from range(n_choices), vectorised skip method."""
    out = np.zeros((count, rf), np.int64)
    taken = []
    for k in range(rf):
        r = rng.integers(0, n_choices - k, size=count, dtype=np.int64)
        if taken:
            srt = np.sort(np.stack(taken, axis=1), axis=1)
            for j in range(srt.shape[1]):
                r = r + (r >= srt[:, j])
        out[:, k] = r
        taken.append(r)
    return out


def _zipf_weights(rng, n):
    r = rng.uniform(1.0, 1e6, size=n)
    return r ** -1.1


def topic_names(n):
    return ["t%05d" % (i // 100) for i in range(n)]


def partition_ids(n):
    return np.arange(n, dtype=np.int64) % 100


def make_cluster(P, B, rf=3, weights="uniform", nsets=0, set_size=0, seed=0, with_names=False,
                 num_replicas=None, broker_hi=None):
    """Generic generator.  weights: 'uniform' (absent -> 1.0), 'zipf', 'int' (1..8)."""
    rng = np.random.default_rng(seed)
    if nsets:
        members = np.stack([np.sort(rng.choice(B, size=set_size, replace=False)) + 1
                            for _ in range(nsets)])
        pset = rng.integers(0, nsets, size=P, dtype=np.int64)
        idx = _distinct(rng, set_size, P, rf)
        reps = members[pset[:, None], idx]
        set_ids = members.reshape(-1)
        set_off = np.arange(nsets + 1, dtype=np.int64) * set_size
        set_idx = pset
    else:
        hi = broker_hi or B
        reps = _distinct(rng, hi, P, rf) + 1
        set_ids = set_off = set_idx = None
    if weights == "uniform":
        w = np.zeros(P)
    elif weights == "zipf":
        w = _zipf_weights(rng, P)
    elif weights == "int":
        w = rng.integers(1, 9, size=P).astype(np.float64)
    else:
        raise ValueError(weights)
    off = np.arange(P + 1, dtype=np.int64) * rf
    nr = np.zeros(P, np.int64) if num_replicas is None else num_replicas
    names = topic_names(P) if with_names else None
    pids = partition_ids(P) if with_names else None
    return ClusterSoA(reps.reshape(-1), off, w, nr, set_ids, set_off, set_idx, None, names, pids)


# c3nl: BASELINE.json configs[2]'s cluster without -allow-leader (MoveNonLeaders at 1M x 1000
# with 256 allowed sets of 64: the 2-slot scan the headline's leader 2-cycle never reaches);
# w16k: the engine's widest broker universe (1M partitions x 16384 brokers, Zipf, auto lists)
SEEDS = {"c2": 0x5EED0002, "c3": 0x5EED0003, "c3nl": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005,
         "w16k": 0x5EED0016}
WORKLOADS = tuple(SEEDS)


def config(name, scale=1.0, seed=None, with_names=False):
    """BASELINE.json configs c2..c5 (optionally scaled down in partitions), c3nl, w16k."""
    base = {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2,
            "min_unbalance": 0.01, "brokers": None}
    s = seed if seed is not None else SEEDS[name]
    if name == "c2":
        P = max(1, int(10000 * scale))
        cl = make_cluster(P, 50, 3, "uniform", seed=s, with_names=with_names)
        cfg = dict(base, min_unbalance=0.0)
        return cl, cfg, {"workload": "c2", "partitions": P, "brokers": 50, "rf": 3,
                         "weights": "uniform", "max_reassign": 100}
    if name == "c3":
        P = max(1, int(1_000_000 * scale))
        cl = make_cluster(P, 1000, 3, "zipf", nsets=256, set_size=64, seed=s, with_names=with_names)
        cfg = dict(base, allow_leader=True, min_unbalance=0.0)
        return cl, cfg, {"workload": "c3", "partitions": P, "brokers": 1000, "rf": 3,
                         "weights": "zipf", "allowed_sets": "256x64", "allow_leader": True,
                         "max_reassign": 1000}
    if name == "c3nl":
        P = max(1, int(1_000_000 * scale))
        cl = make_cluster(P, 1000, 3, "zipf", nsets=256, set_size=64, seed=s, with_names=with_names)
        cfg = dict(base, min_unbalance=0.0)
        return cl, cfg, {"workload": "c3nl", "partitions": P, "brokers": 1000, "rf": 3,
                         "weights": "zipf", "allowed_sets": "256x64", "allow_leader": False,
                         "max_reassign": 1000}
    if name == "w16k":
        P = max(1, int(1_000_000 * scale))
        cl = make_cluster(P, 16384, 3, "zipf", seed=s, with_names=with_names)
        cfg = dict(base, min_unbalance=0.0)
        return cl, cfg, {"workload": "w16k", "partitions": P, "brokers": 16384, "rf": 3,
                         "weights": "zipf", "max_reassign": 1000}
    if name == "c4":
        P = max(1, int(1_000_000 * scale))
        rng = np.random.default_rng(s + 1)
        nr = np.zeros(P, np.int64)
        k = min(300, P // 4)
        pick = rng.choice(P, size=2 * k, replace=False)
        nr[pick[:k]] = 2
        nr[pick[k:]] = 4
        cl = make_cluster(P, 1000, 3, "zipf", seed=s, with_names=with_names, num_replicas=nr)
        brokers = [b for b in range(1, 1201) if not (951 <= b <= 1000)]
        cfg = dict(base, min_unbalance=0.0, brokers=brokers)
        return cl, cfg, {"workload": "c4", "partitions": P, "brokers": "1000->1150 allowed",
                         "rf": 3, "weights": "zipf", "remove": k, "add": k, "max_reassign": 1000}
    if name == "c5":
        P = max(1, int(10_000_000 * scale))
        cl = make_cluster(P, 4096, 3, "zipf", seed=s, with_names=with_names)
        cfg = dict(base, min_unbalance=0.0)
        return cl, cfg, {"workload": "c5", "partitions": P, "brokers": 4096, "rf": 3,
                         "weights": "zipf", "max_reassign": 1000}
    raise ValueError(name)


def to_plist(cl):
    """ClusterSoA -> reference JSON dict form (small clusters only)."""
    parts = []
    names = cl.topics or topic_names(cl.n)
    pids = cl.partition_ids if cl.partition_ids is not None else partition_ids(cl.n)
    for i in range(cl.n):
        p = {"topic": names[i], "partition": int(pids[i]),
             "replicas": cl.replica_ids[cl.replica_off[i]:cl.replica_off[i + 1]].tolist()}
        if cl.weight[i] != 0:
            p["weight"] = float(cl.weight[i])
        if cl.num_replicas[i] != 0:
            p["num_replicas"] = int(cl.num_replicas[i])
        if cl.set_idx[i] >= 0:
            s = cl.set_idx[i]
            p["brokers"] = cl.set_ids[cl.set_off[s]:cl.set_off[s + 1]].tolist()
        if cl.num_consumers[i] != 0:
            p["num_consumers"] = int(cl.num_consumers[i])
        parts.append(p)
    return {"version": 1, "partitions": parts}
