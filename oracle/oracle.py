"""ctypes binding of the CPU oracle (oracle/kb_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product (kafkabalancer_amd/).

The partition-list dict form used throughout the tests mirrors the reference
JSON (kafkabalancer.go:40-58):
    {"version": 1, "partitions": [{"topic": str, "partition": int,
      "replicas": [int] | None, "weight": float, "num_replicas": int,
      "brokers": [int] | None, "num_consumers": int}, ...]}
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libkboracle.so")

SEM_GO = 0
SEM_APPLIED = 1
STEP_NAMES = ["ValidateWeights", "ValidateReplicas", "FillDefaults", "RemoveExtraReplicas",
              "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders",
              "MoveLeaders", "MoveNonLeaders"]
KIND_NAMES = {0: "none", 1: "replace", 2: "remove", 3: "add", 4: "swap"}


class _Slice(C.Structure):
    _fields_ = [("a", C.POINTER(C.c_int64)), ("len", C.c_int64), ("cap", C.c_int64)]


class _Part(C.Structure):
    _fields_ = [("topic", C.c_char_p), ("partition", C.c_int64), ("replicas", _Slice),
                ("weight", C.c_double), ("num_replicas", C.c_int64), ("brokers", _Slice),
                ("num_consumers", C.c_int64)]


class _PL(C.Structure):
    _fields_ = [("version", C.c_int64), ("parts", C.POINTER(_Part)), ("n", C.c_int64)]


class _Cfg(C.Structure):
    _fields_ = [("allow_leader", C.c_int), ("rebalance_leaders", C.c_int),
                ("min_replicas", C.c_int64), ("min_unbalance", C.c_double),
                ("complete_partition", C.c_int), ("brokers", C.POINTER(C.c_int64)),
                ("nbrokers", C.c_int64), ("brokers_nil", C.c_int)]


class _Res(C.Structure):
    _fields_ = [("status", C.c_int), ("step", C.c_int), ("pidx", C.c_int64), ("kind", C.c_int),
                ("from_", C.c_int64), ("to", C.c_int64), ("slot", C.c_int64), ("part", _Part),
                ("su", C.c_double), ("cu", C.c_double), ("err", C.c_char * 1024)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        L.or_plist_build.restype = P(_PL)
        L.or_plist_build.argtypes = [C.c_int64, C.c_char_p, P(C.c_int64), P(C.c_int64),
                                     P(C.c_int64), P(C.c_int64), P(C.c_int8), P(C.c_double),
                                     P(C.c_int64), C.c_int64, P(C.c_int64), P(C.c_int64),
                                     P(C.c_int64), P(C.c_int64)]
        L.or_balance.argtypes = [P(_PL), P(_Cfg), C.c_int, P(_Res)]
        L.or_balance.restype = C.c_int
        L.or_step.argtypes = [P(_PL), P(_Cfg), C.c_int, C.c_uint, P(_Res)]
        L.or_step.restype = C.c_int
        L.or_run_plan.argtypes = [P(_PL), P(_Cfg), C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int,
                                  P(C.c_void_p), C.c_char_p, C.c_size_t, P(C.c_int64)]
        L.or_run_plan.restype = C.c_int
        L.or_move_sample.argtypes = [P(_PL), P(_Cfg), C.c_int, C.c_int64, P(C.c_double)]
        L.or_move_sample.restype = C.c_int64
        L.or_plist_replicas.argtypes = [P(_PL), C.c_int64, P(C.c_int64), C.c_int64]
        L.or_plist_replicas.restype = C.c_int64
        L.or_unbalance.argtypes = [P(C.c_double), C.c_int64]
        L.or_unbalance.restype = C.c_double
        L.or_format_float.argtypes = [C.c_double, C.c_char_p]
        L.or_free.argtypes = [C.c_void_p]
        L.or_set_threads.argtypes = [C.c_int]
        L.or_set_threads.restype = None
        L.or_set_window.argtypes = [C.c_int]
        L.or_set_window.restype = None
        L.or_walk_stops.argtypes = []
        L.or_walk_stops.restype = C.c_int64
        L.or_reset_walk_stops.argtypes = []
        L.or_reset_walk_stops.restype = None
        _lib = L
    return _lib


def build():
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _i64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(C.POINTER(C.c_int64))


class OraclePL:
    """A partition list living in oracle (C) memory."""

    def __init__(self, plist):
        parts = plist["partitions"]
        n = len(parts)
        topics = [p["topic"].encode() for p in parts]
        toff = np.zeros(n + 1, np.int64)
        toff[1:] = np.cumsum([len(t) for t in topics])
        blob = b"".join(topics)
        reps = [p.get("replicas") for p in parts]
        roff = np.zeros(n + 1, np.int64)
        roff[1:] = np.cumsum([len(r) if r else 0 for r in reps])
        rflat = np.array([b for r in reps if r for b in r], np.int64)
        rnil = np.array([1 if r is None else 0 for r in reps], np.int8)
        w = np.array([float(p.get("weight", 0) or 0) for p in parts], np.float64)
        nr = np.array([int(p.get("num_replicas", 0) or 0) for p in parts], np.int64)
        nc = np.array([int(p.get("num_consumers", 0) or 0) for p in parts], np.int64)
        sets, sidx = {}, np.full(n, -1, np.int64)
        for i, p in enumerate(parts):
            b = p.get("brokers")
            if b is None:
                continue
            key = tuple(b)
            if key not in sets:
                sets[key] = len(sets)
            sidx[i] = sets[key]
        slist = sorted(sets, key=sets.get)
        soff = np.zeros(len(slist) + 1, np.int64)
        soff[1:] = np.cumsum([len(s) for s in slist])
        sflat = np.array([b for s in slist for b in s], np.int64)
        self._init_arrays(n, blob, toff, np.array([p["partition"] for p in parts], np.int64),
                          rflat, roff, rnil, w, nr, len(slist), sflat, soff, sidx, nc)

    @classmethod
    def from_soa(cls, topics_blob, topic_off, partition, rep_flat, rep_off, weight, num_replicas,
                 set_flat, set_off, set_idx, num_consumers):
        self = cls.__new__(cls)
        n = len(partition)
        self._init_arrays(n, topics_blob, topic_off, partition, rep_flat, rep_off, None, weight,
                          num_replicas, len(set_off) - 1, set_flat, set_off, set_idx, num_consumers)
        return self

    def _init_arrays(self, n, blob, toff, part, rflat, roff, rnil, w, nr, nsets, sflat, soff, sidx, nc):
        L = lib()
        keep = []

        def p64(a):
            a, p = _i64(a)
            keep.append(a)
            return p
        w = np.ascontiguousarray(w, np.float64)
        keep.append(w)
        rnil_p = None
        if rnil is not None:
            rnil = np.ascontiguousarray(rnil, np.int8)
            keep.append(rnil)
            rnil_p = rnil.ctypes.data_as(C.POINTER(C.c_int8))
        if len(rflat) == 0:
            rflat = np.zeros(1, np.int64)
        if len(sflat) == 0:
            sflat = np.zeros(1, np.int64)
        self.pl = L.or_plist_build(n, blob, p64(toff), p64(part), p64(rflat), p64(roff), rnil_p,
                                   w.ctypes.data_as(C.POINTER(C.c_double)), p64(nr), nsets,
                                   p64(sflat), p64(soff), p64(sidx), p64(nc))
        self.n = n

    def replicas(self, i):
        buf = (C.c_int64 * 64)()
        k = lib().or_plist_replicas(self.pl, i, buf, 64)
        return [buf[j] for j in range(k)]

    def state(self):
        return [self.replicas(i) for i in range(self.n)]

    def partition(self, i):
        p = self.pl.contents.parts[i]
        return _part_to_dict(p)


def _slice_list(s):
    if not s.a:
        return None
    return [s.a[k] for k in range(s.len)]


def _part_to_dict(p):
    return {"topic": p.topic.decode(), "partition": p.partition, "replicas": _slice_list(p.replicas),
            "weight": p.weight, "num_replicas": p.num_replicas, "brokers": _slice_list(p.brokers),
            "num_consumers": p.num_consumers}


def make_cfg(cfg):
    """cfg dict: allow_leader, rebalance_leaders, min_replicas, min_unbalance,
    complete_partition, brokers (None = nil)."""
    c = _Cfg()
    c.allow_leader = int(bool(cfg.get("allow_leader", False)))
    c.rebalance_leaders = int(bool(cfg.get("rebalance_leaders", False)))
    c.min_replicas = int(cfg.get("min_replicas", 2))
    c.min_unbalance = float(cfg.get("min_unbalance", 0.01))
    c.complete_partition = int(bool(cfg.get("complete_partition", True)))
    b = cfg.get("brokers")
    if b is None:
        c.brokers_nil = 1
        c.nbrokers = 0
        c._keep = None
    else:
        arr = (C.c_int64 * max(1, len(b)))(*b)
        c.brokers = C.cast(arr, C.POINTER(C.c_int64))
        c.nbrokers = len(b)
        c.brokers_nil = 0
        c._keep = arr
    return c


def default_cfg():
    """DefaultRebalanceConfig (balancer.go:24-32)."""
    return {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2,
            "min_unbalance": 0.01, "complete_partition": True, "brokers": None}


def balance(opl, cfg, sem=SEM_GO):
    """One Balance() call (balancer.go:49-65) on an OraclePL (mutates it)."""
    res = _Res()
    c = make_cfg(cfg)
    lib().or_balance(opl.pl, C.byref(c), sem, C.byref(res))
    out = {"status": res.status, "step": STEP_NAMES[res.step] if res.status else None,
           "err": res.err.decode() if res.status < 0 else None}
    if res.status == 1:
        out.update(pidx=res.pidx, kind=KIND_NAMES[res.kind], from_=res.from_, to=res.to,
                   slot=res.slot, partition=_part_to_dict(res.part), su=res.su, cu=res.cu)
    return out


def step(opl, cfg, mask, sem=SEM_GO):
    """Balance() over the steps whose bit is set in mask (bit k = STEP_NAMES[k]) only."""
    res = _Res()
    c = make_cfg(cfg)
    lib().or_step(opl.pl, C.byref(c), sem, mask, C.byref(res))
    out = {"status": res.status, "step": STEP_NAMES[res.step] if res.status else None,
           "err": res.err.decode() if res.status < 0 else None}
    if res.status == 1:
        out.update(pidx=res.pidx, kind=KIND_NAMES[res.kind], from_=res.from_, to=res.to,
                   slot=res.slot, partition=_part_to_dict(res.part), su=res.su, cu=res.cu)
    return out


def run_plan(opl, cfg, max_reassign=1, complete_partition=True, full_output=False, unique=False,
             sem=SEM_GO):
    """run()'s main loop + output (kafkabalancer.go:177-241). Returns (code, out_bytes, err)."""
    out = C.c_void_p()
    err = C.create_string_buffer(2048)
    nsteps = C.c_int64()
    c = make_cfg(cfg)
    code = lib().or_run_plan(opl.pl, C.byref(c), max_reassign, int(complete_partition),
                             int(full_output), int(unique), sem, C.byref(out), err, 2048,
                             C.byref(nsteps))
    data = b""
    if out.value:
        data = C.string_at(out.value)
        lib().or_free(out)
    return code, data, err.value.decode()


def move_sample(opl, cfg, leaders, max_parts):
    cu = C.c_double()
    n = lib().or_move_sample(opl.pl, C.byref(make_cfg(cfg)), int(leaders), max_parts, C.byref(cu))
    return n, cu.value


def set_threads(n):
    """Worker threads of the oracle's move() (identical results for any n)."""
    lib().or_set_threads(int(n))


def walk_stops(reset=False):
    """Target walks the windowed search's early stop ended since the last reset (its n >= 64
    branch, kb_oracle.c move_window)."""
    n = int(lib().or_walk_stops())
    if reset:
        lib().or_reset_walk_stops()
    return n


def set_window(on):
    """Golden generation only: move()'s windowed exact search (same results as the literal
    loop, kb_oracle.c move_window)."""
    lib().or_set_window(int(bool(on)))


def format_float(x):
    buf = C.create_string_buffer(64)
    lib().or_format_float(x, buf)
    return buf.value.decode()


def unbalance(loads):
    a = np.ascontiguousarray(loads, np.float64)
    return lib().or_unbalance(a.ctypes.data_as(C.POINTER(C.c_double)), len(a))
