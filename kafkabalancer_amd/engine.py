"""ctypes binding of libkbengine.so (the C ABI in include/kbengine.h).

This is the same binding a cgo shim would make: plain
pointers and sizes.  There is no CPU fallback: if the HIP library is missing
or no GPU is visible, constructing an Engine raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KB_ENGINE_LIB") or os.path.join(_HERE, "lib", "libkbengine.so")

KB_NOCHANGE, KB_CHANGE, KB_RETRY, KB_GROW = 0, 1, 2, 3
KB_SEM_APPLIED, KB_SEM_GO = 0, 1
ERRORS = {-1: "KB_ERR_INVALID", -2: "KB_ERR_HIP", -3: "KB_ERR_UNSUPPORTED", -4: "KB_ERR_STEP",
          -5: "KB_ERR_CAPACITY", -6: "KB_ERR_PANIC"}
STEP_NAMES = ["ValidateWeights", "ValidateReplicas", "FillDefaults", "RemoveExtraReplicas",
              "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders", "MoveLeaders",
              "MoveNonLeaders"]
KIND_NAMES = {0: "none", 1: "replace", 2: "remove", 3: "add", 4: "swap"}
KB_STEPS_ALL = 0x1FF

EXPORTS = ["kb_abi_version", "kb_engine_create", "kb_engine_balance", "kb_engine_plan",
           "kb_engine_replicas", "kb_engine_loads", "kb_engine_unbalance", "kb_engine_stats",
           "kb_engine_timings", "kb_engine_set_timing", "kb_engine_stamps", "kb_engine_bench_scan", "kb_engine_bench_step",
           "kb_engine_last_error", "kb_engine_destroy", "kb_engine_summary_bytes",
           "kb_engine_step_begin", "kb_engine_step_finish", "kb_engine_set_stream",
           "kb_engine_sharded_reset", "kb_engine_sharded_scan", "kb_engine_sharded_resolve",
           "kb_engine_sharded_collect", "kb_engine_set_incremental", "kb_engine_step",
           "kb_engine_host_timings", "kb_comm_unique_id", "kb_engine_comm_init", "kb_engine_sharded_plan",
           "kb_set_diagnostics", "kb_diagnostics_enabled", "kb_engine_plan_until"]

P64 = C.POINTER(C.c_int64)
PD = C.POINTER(C.c_double)


class kb_cluster(C.Structure):
    _fields_ = [("n_partitions", C.c_int64), ("replica_ids", P64), ("replica_off", P64),
                ("weight", PD), ("num_replicas", P64), ("num_consumers", P64),
                ("n_sets", C.c_int64), ("set_ids", P64), ("set_off", P64), ("set_idx", P64),
                ("topic_blob", C.c_char_p), ("topic_off", P64), ("partition_id", P64)]


class kb_config(C.Structure):
    _fields_ = [("allow_leader", C.c_int32), ("rebalance_leaders", C.c_int32),
                ("min_replicas", C.c_int64), ("min_unbalance", C.c_double),
                ("brokers", P64), ("n_brokers", C.c_int64), ("brokers_nil", C.c_int32),
                ("semantics", C.c_int32), ("device", C.c_int32), ("list_slack", C.c_int32),
                ("shard_begin", C.c_int64), ("shard_end", C.c_int64),
                ("exact_unbalance", C.c_int32), ("time_kernels", C.c_int32)]


class kb_change(C.Structure):
    _fields_ = [("status", C.c_int32), ("step", C.c_int32), ("kind", C.c_int32), ("slot", C.c_int32),
                ("partition", C.c_int64), ("from_broker", C.c_int64), ("to_broker", C.c_int64),
                ("unbalance_before", C.c_double), ("unbalance_after", C.c_double),
                ("exact", C.c_int32), ("err_code", C.c_int32), ("err_broker", C.c_int64)]


class kb_stats(C.Structure):
    _fields_ = [("steps", C.c_int64), ("candidates", C.c_int64), ("contenders", C.c_int64),
                ("exact_folds", C.c_int64), ("scan_bytes", C.c_int64), ("device_ms", C.c_double),
                ("n_brokers", C.c_int64), ("n_sets", C.c_int64), ("integral", C.c_int32),
                ("max_replicas", C.c_int32), ("refreshes", C.c_int64), ("exact_halts", C.c_int64),
                ("scan_workgroups", C.c_int64), ("retries", C.c_int64), ("spill_grows", C.c_int64),
                ("blocks_scanned", C.c_int64), ("relists", C.c_int64),
                ("fused_pairs", C.c_int64), ("fused_summaries", C.c_int64),
                ("eager", C.c_int64), ("eager_switches", C.c_int64), ("fast_preps", C.c_int64)]


_lib = None


def lib():
    """Load libkbengine.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libkbengine.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.kb_abi_version.restype = C.c_int
        L.kb_engine_create.argtypes = [C.POINTER(kb_cluster), C.POINTER(kb_config), C.POINTER(vp)]
        L.kb_engine_create.restype = C.c_int
        L.kb_engine_balance.argtypes = [vp, C.POINTER(kb_change)]
        L.kb_engine_balance.restype = C.c_int
        L.kb_engine_step.argtypes = [vp, C.c_uint32, C.POINTER(kb_change)]
        L.kb_engine_step.restype = C.c_int
        L.kb_engine_plan.argtypes = [vp, C.c_int64, C.POINTER(kb_change), P64]
        L.kb_engine_plan.restype = C.c_int
        L.kb_engine_replicas.argtypes = [vp, C.c_int64, P64, C.c_int64]
        L.kb_engine_replicas.restype = C.c_int64
        L.kb_engine_loads.argtypes = [vp, P64, PD, C.c_int64]
        L.kb_engine_loads.restype = C.c_int64
        L.kb_engine_unbalance.argtypes = [vp]
        L.kb_engine_unbalance.restype = C.c_double
        L.kb_engine_stats.argtypes = [vp, C.POINTER(kb_stats)]
        L.kb_engine_stats.restype = C.c_int
        L.kb_engine_timings.argtypes = [vp, PD, P64, C.c_int]
        L.kb_engine_timings.restype = C.c_int
        if hasattr(L, "kb_engine_host_timings"):        # (diagnostic; older builds in A/B runs lack it)
            L.kb_engine_host_timings.argtypes = [vp, PD, C.c_int]
            L.kb_engine_host_timings.restype = C.c_int
        L.kb_engine_set_timing.argtypes = [vp, C.c_int32]
        L.kb_engine_set_timing.restype = C.c_int
        L.kb_engine_stamps.argtypes = [vp, P64, C.c_int]
        L.kb_engine_stamps.restype = C.c_int
        L.kb_engine_bench_scan.argtypes = [vp, C.c_int, PD]
        L.kb_engine_bench_scan.restype = C.c_int
        if hasattr(L, "kb_engine_bench_step"):          # (diagnostic; older builds in A/B runs lack it)
            L.kb_engine_bench_step.argtypes = [vp, C.c_int, PD]
            L.kb_engine_bench_step.restype = C.c_int
        L.kb_engine_last_error.argtypes = [vp, C.c_char_p, C.c_size_t]
        L.kb_engine_last_error.restype = C.c_int
        L.kb_engine_destroy.argtypes = [vp]
        L.kb_engine_destroy.restype = None
        L.kb_engine_summary_bytes.argtypes = [vp]
        L.kb_engine_summary_bytes.restype = C.c_int64
        L.kb_engine_step_begin.argtypes = [vp, vp]
        L.kb_engine_step_begin.restype = C.c_int
        L.kb_engine_step_finish.argtypes = [vp, vp, C.c_int32, C.POINTER(kb_change)]
        L.kb_engine_step_finish.restype = C.c_int
        L.kb_engine_set_stream.argtypes = [vp, vp]
        L.kb_engine_set_stream.restype = C.c_int
        L.kb_engine_sharded_reset.argtypes = [vp, C.c_int64]
        L.kb_engine_sharded_reset.restype = C.c_int
        L.kb_engine_sharded_scan.argtypes = [vp, vp]
        L.kb_engine_sharded_scan.restype = C.c_int
        L.kb_engine_sharded_resolve.argtypes = [vp, vp, C.c_int32]
        L.kb_engine_sharded_resolve.restype = C.c_int
        L.kb_engine_sharded_collect.argtypes = [vp, C.POINTER(kb_change), C.c_int64, P64]
        L.kb_engine_sharded_collect.restype = C.c_int
        if hasattr(L, "kb_engine_debug_records"):       # (diagnostic)
            L.kb_engine_debug_records.argtypes = [vp, vp, C.c_int64]
            L.kb_engine_debug_records.restype = C.c_int64
        if hasattr(L, "kb_engine_ctl_scalars"):         # (diagnostic)
            L.kb_engine_ctl_scalars.argtypes = [vp, PD, C.c_int]
            L.kb_engine_ctl_scalars.restype = C.c_int
        if hasattr(L, "kb_engine_sharded_plan"):        # (ABI 9; older builds in A/B runs lack it)
            L.kb_comm_unique_id.argtypes = [C.c_char_p]
            L.kb_comm_unique_id.restype = C.c_int
            L.kb_engine_comm_init.argtypes = [vp, C.c_int32, C.c_int32, C.c_char_p]
            L.kb_engine_comm_init.restype = C.c_int
            L.kb_engine_sharded_plan.argtypes = [vp, C.c_int64, C.POINTER(kb_change), P64]
            L.kb_engine_sharded_plan.restype = C.c_int
        any_abi = os.environ.get("KB_ABI_ANY") == "1"      # diagnostic: older builds (bisecting)
        if hasattr(L, "kb_engine_set_incremental"):
            L.kb_engine_set_incremental.argtypes = [vp, C.c_int32]
            L.kb_engine_set_incremental.restype = C.c_int
        if L.kb_abi_version() != 11 and not any_abi:
            raise ImportError("libkbengine.so ABI mismatch")
        # the library's A/B and diagnostic switches (KB_FUSE, KB_EAGER, ...) are read from the
        # environment only after this opt-in (include/kbengine.h); the tests and the bench
        # scripts set KB_DIAGNOSTICS=1, a plain import leaves them off
        if hasattr(L, "kb_set_diagnostics"):
            L.kb_set_diagnostics.argtypes = [C.c_int]
            L.kb_set_diagnostics(1 if os.environ.get("KB_DIAGNOSTICS") == "1" else 0)
        _lib = L
    return _lib


KB_COMM_ID_BYTES = 128


def comm_unique_id():
    """RCCL unique id (rank 0; the caller broadcasts the bytes): kb_comm_unique_id."""
    buf = C.create_string_buffer(KB_COMM_ID_BYTES)
    rc = lib().kb_comm_unique_id(buf)
    if rc != 0:
        raise EngineError(rc, "kb_comm_unique_id failed (%s)" % ERRORS.get(rc, rc))
    return buf.raw


class EngineError(RuntimeError):
    def __init__(self, code, msg, change=None):
        super().__init__(msg)
        self.code = code
        self.change = change


class ClusterSoA:
    """Flat arrays of a PartitionList (kafkabalancer.go:40-58) in the kb_cluster layout."""

    def __init__(self, replica_ids, replica_off, weight, num_replicas, set_ids=None, set_off=None,
                 set_idx=None, num_consumers=None, topics=None, partition_ids=None):
        self.replica_ids = np.ascontiguousarray(replica_ids, np.int64)
        self.replica_off = np.ascontiguousarray(replica_off, np.int64)
        self.n = len(self.replica_off) - 1
        self.weight = np.ascontiguousarray(weight, np.float64)
        self.num_replicas = np.ascontiguousarray(num_replicas, np.int64)
        self.num_consumers = (np.zeros(self.n, np.int64) if num_consumers is None
                              else np.ascontiguousarray(num_consumers, np.int64))
        if set_off is None:
            self.set_ids = np.zeros(1, np.int64)
            self.set_off = np.zeros(1, np.int64)
            self.set_idx = np.full(self.n, -1, np.int64)
        else:
            self.set_ids = np.ascontiguousarray(set_ids if len(set_ids) else [0], np.int64)
            self.set_off = np.ascontiguousarray(set_off, np.int64)
            self.set_idx = np.ascontiguousarray(set_idx, np.int64)
        self.topics = topics
        self.partition_ids = (None if partition_ids is None
                              else np.ascontiguousarray(partition_ids, np.int64))

    @classmethod
    def from_plist(cls, plist):
        """Build from the reference JSON dict form."""
        parts = plist["partitions"] if isinstance(plist, dict) else plist
        reps = [p.get("replicas") or [] for p in parts]
        off = np.zeros(len(parts) + 1, np.int64)
        off[1:] = np.cumsum([len(r) for r in reps])
        flat = np.array([b for r in reps for b in r], np.int64)
        sets, sidx = {}, np.full(len(parts), -1, np.int64)
        for i, p in enumerate(parts):
            b = p.get("brokers")
            if b is None:
                continue
            key = tuple(b)
            sidx[i] = sets.setdefault(key, len(sets))
        slist = sorted(sets, key=sets.get)
        soff = np.zeros(len(slist) + 1, np.int64)
        soff[1:] = np.cumsum([len(s) for s in slist])
        sflat = np.array([b for s in slist for b in s], np.int64)
        return cls(flat, off, [float(p.get("weight", 0) or 0) for p in parts],
                   [int(p.get("num_replicas", 0) or 0) for p in parts], sflat, soff, sidx,
                   [int(p.get("num_consumers", 0) or 0) for p in parts],
                   [p["topic"] for p in parts], [int(p["partition"]) for p in parts])

    def to_struct(self):
        c = kb_cluster()
        c.n_partitions = self.n
        c.replica_ids = self.replica_ids.ctypes.data_as(P64) if len(self.replica_ids) else \
            np.zeros(1, np.int64).ctypes.data_as(P64)
        c.replica_off = self.replica_off.ctypes.data_as(P64)
        c.weight = self.weight.ctypes.data_as(PD)
        c.num_replicas = self.num_replicas.ctypes.data_as(P64)
        c.num_consumers = self.num_consumers.ctypes.data_as(P64)
        c.n_sets = len(self.set_off) - 1
        c.set_ids = self.set_ids.ctypes.data_as(P64)
        c.set_off = self.set_off.ctypes.data_as(P64)
        c.set_idx = self.set_idx.ctypes.data_as(P64)
        self._keep = []
        if self.topics is not None:
            enc = [t.encode() for t in self.topics]
            toff = np.zeros(self.n + 1, np.int64)
            toff[1:] = np.cumsum([len(t) for t in enc])
            blob = b"".join(enc)
            self._keep += [blob, toff]
            c.topic_blob = blob
            c.topic_off = toff.ctypes.data_as(P64)
        if self.partition_ids is not None:
            c.partition_id = self.partition_ids.ctypes.data_as(P64)
        return c


def _change_dict(ch):
    return {"status": ch.status, "step": STEP_NAMES[ch.step] if 0 <= ch.step < 9 else None,
            "kind": KIND_NAMES.get(ch.kind, "?"), "slot": ch.slot, "pidx": ch.partition,
            "from_": ch.from_broker, "to": ch.to_broker, "su": ch.unbalance_before,
            "cu": ch.unbalance_after, "exact": ch.exact}


class Engine:
    """One device-resident engine over a cluster (kb_engine_*)."""

    def __init__(self, cluster, cfg, semantics=KB_SEM_APPLIED, device=0, shard=None, list_slack=0,
                 exact_unbalance=False, time_kernels=False, incremental=False):
        L = lib()
        self._cap = 1024                  # plan_raw's change buffer (grown by doubling)
        self._buf = (kb_change * self._cap)()
        if not isinstance(cluster, ClusterSoA):
            cluster = ClusterSoA.from_plist(cluster)
        self.cluster = cluster
        cs = cluster.to_struct()
        kc = kb_config()
        kc.allow_leader = int(bool(cfg.get("allow_leader", False)))
        kc.rebalance_leaders = int(bool(cfg.get("rebalance_leaders", False)))
        kc.min_replicas = int(cfg.get("min_replicas", 2))
        kc.min_unbalance = float(cfg.get("min_unbalance", 0.01))
        b = cfg.get("brokers")
        if b is None:
            kc.brokers_nil = 1
            self._brokers = np.zeros(1, np.int64)
            kc.n_brokers = 0
        else:
            self._brokers = np.ascontiguousarray(b if len(b) else [0], np.int64)
            kc.n_brokers = len(b)
            kc.brokers_nil = 0
        kc.brokers = self._brokers.ctypes.data_as(P64)
        kc.semantics = semantics
        kc.device = device
        kc.list_slack = list_slack
        kc.exact_unbalance = int(bool(exact_unbalance))
        kc.time_kernels = int(bool(time_kernels))
        if shard is not None:
            kc.shard_begin, kc.shard_end = shard
        h = C.c_void_p()
        rc = L.kb_engine_create(C.byref(cs), C.byref(kc), C.byref(h))
        self.h = h
        if rc < 0:
            msg = self.last_error() if h.value else "kb_engine_create failed"
            self.close()
            raise EngineError(rc, "%s: %s" % (ERRORS.get(rc, rc), msg))
        if incremental:
            try:
                self.set_incremental(True)
            except EngineError:
                self.close()          # (the handle created above: no leaked device memory)
                raise

    def set_incremental(self, on):
        """Incremental rescoring mode: scans read only the partition blocks
        a lower-bound certificate cannot exclude; same results as the full scan."""
        rc = lib().kb_engine_set_incremental(self.h, int(bool(on)))
        if rc != 0:
            raise EngineError(rc, self.last_error())

    def last_error(self):
        buf = C.create_string_buffer(4096)
        lib().kb_engine_last_error(self.h, buf, 4096)
        return buf.value.decode()

    def balance(self):
        """One Balance() step; returns the change dict, None for no change; raises EngineError."""
        ch = kb_change()
        rc = lib().kb_engine_balance(self.h, C.byref(ch))
        if rc == KB_NOCHANGE:
            return None
        if rc == KB_CHANGE:
            return _change_dict(ch)
        raise EngineError(rc, self.last_error(), _change_dict(ch))

    def step(self, mask):
        """One Balance() restricted to the steps in `mask` (bit k = STEP_NAMES[k]; a name or a
        list of names also works): the change dict, None for no change; raises EngineError."""
        if isinstance(mask, str):
            mask = [mask]
        if not isinstance(mask, int):
            bits = 0
            for n in mask:
                if n not in STEP_NAMES:
                    raise ValueError("unknown step %r" % (n,))
                bits |= 1 << STEP_NAMES.index(n)      # (a repeated name sets its bit once)
            mask = bits
        if not 0 <= mask <= KB_STEPS_ALL:
            raise ValueError("step mask %#x outside the steps table (0..%#x)" % (mask, KB_STEPS_ALL))
        ch = kb_change()
        rc = lib().kb_engine_step(self.h, mask, C.byref(ch))
        if rc == KB_NOCHANGE:
            return None
        if rc == KB_CHANGE:
            return _change_dict(ch)
        raise EngineError(rc, self.last_error(), _change_dict(ch))

    def plan(self, max_steps):
        """Device-resident plan; returns (changes, error_or_None)."""
        return self.changes(*self.plan_raw(max_steps))

    def plan_raw(self, max_steps):
        """The plan call alone (the bench's timed region): (kb_change buffer, n, rc).  The
        buffer is the engine's own and is reused by the next plan_raw: read it (changes())
        first.  (A ctypes array type of a new length costs 15-25 us to create, so the
        buffer keeps one type per capacity and grows by doubling.)"""
        if max_steps > self._cap:
            while self._cap < max_steps:
                self._cap *= 2
            self._buf = (kb_change * self._cap)()
        n = C.c_int64()
        rc = lib().kb_engine_plan(self.h, max_steps, self._buf, C.byref(n))
        return self._buf, n.value, rc

    def changes(self, buf, n, rc):
        """plan_raw's result as (changes, error_or_None)."""
        changes = [_change_dict(buf[i]) for i in range(n)]
        err = None
        if rc < 0:
            err = EngineError(rc, self.last_error(), changes[-1] if changes else None)
            changes = changes[:-1]
        elif changes and changes[-1]["status"] == KB_NOCHANGE:
            changes = changes[:-1]
        return changes, err

    def replicas(self, i):
        buf = (C.c_int64 * 32)()
        k = lib().kb_engine_replicas(self.h, i, buf, 32)
        if k < 0:
            raise EngineError(k, self.last_error())
        return [buf[j] for j in range(k)]

    def state(self):
        return [self.replicas(i) for i in range(self.cluster.n)]

    def loads(self):
        n = lib().kb_engine_loads(self.h, None, None, 0)
        ids = np.zeros(max(n, 1), np.int64)
        ld = np.zeros(max(n, 1), np.float64)
        lib().kb_engine_loads(self.h, ids.ctypes.data_as(P64), ld.ctypes.data_as(PD), n)
        return dict(zip(ids[:n].tolist(), ld[:n].tolist()))

    def unbalance(self):
        return lib().kb_engine_unbalance(self.h)

    def stats(self):
        s = kb_stats()
        lib().kb_engine_stats(self.h, C.byref(s))
        return {f: getattr(s, f) for f, _ in s._fields_}

    KERNELS = ("step", "scan", "refresh", "bound", "step_inner", "scan_inner", "pair", "eager", "eager_edit")

    def timings(self):
        """{kernel: (total_ms, launches)} of the plans since set_timing; mode 1: step / scan are
        rocprof-comparable device-clock spans, step_inner / scan_inner first-start..last-end."""
        ms = np.zeros(9)
        n = np.zeros(9, np.int64)
        lib().kb_engine_timings(self.h, ms.ctypes.data_as(PD), n.ctypes.data_as(P64), 9)
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.KERNELS)}

    def set_timing(self, on):
        """Kernel timing for the following plans (resets the sums): False/0 off, True/1
        device clock for k_scan / k_step, 2 HIP events around every launch (dispatch
        included, what rocprofv3 reports)."""
        rc = lib().kb_engine_set_timing(self.h, 2 if on == 2 else int(bool(on)))
        if rc != 0:
            raise EngineError(rc, self.last_error())

    def host_timings(self):
        """Diagnostic: host phases of the plan calls since set_timing (us) and their count."""
        us = np.zeros(5)
        lib().kb_engine_host_timings(self.h, us.ctypes.data_as(PD), 5)
        return {"reset": us[0], "enqueue": us[1], "wait": us[2], "convert": us[3], "calls": int(us[4])}

    def debug_records(self):
        """Diagnostic: the last scan's record headers as a numpy structured array."""
        ct = np.dtype([("s", "<i4"), ("t", "<i4"), ("w", "<f8"), ("iter", "<u8"), ("kind", "<i4"), ("pad", "<i4")])
        dt = np.dtype([("dmin", "<f8", 2), ("cand", "<u8", 2), ("nkeys", "<u4"), ("flags", "<u4"),
                       ("fmask", "<u4"), ("nkk", "<u2", 2), ("best", ct, 2)])
        assert dt.itemsize == 112
        n = lib().kb_engine_debug_records(self.h, None, 0)
        out = np.zeros(max(n, 1), dt)
        lib().kb_engine_debug_records(self.h, out.ctypes.data_as(C.c_void_p), n)
        return out[:n]

    def ctl_scalars(self):
        """Diagnostic: the control block's scalars for the next step (ub per kind, eps, U0, V,
        avg, r range, E, S)."""
        v = np.zeros(10)
        lib().kb_engine_ctl_scalars(self.h, v.ctypes.data_as(PD), 10)
        return dict(zip(("ub0", "ub1", "eps", "U0", "V", "avg", "rlo", "rhi", "E", "S"), v.tolist()))

    def stamps(self):
        """Diagnostic build only: accumulated phase ticks (100 MHz) of the k_step phases."""
        out = np.zeros(32, np.int64)
        lib().kb_engine_stamps(self.h, out.ctypes.data_as(P64), 32)
        return out.tolist()

    def bench_step(self, iters=100):
        """Diagnostic: k_step alone on a fixed input (us per launch; phase costs from -DKB_STOP_AT builds)."""
        v = C.c_double()
        rc = lib().kb_engine_bench_step(self.h, iters, C.byref(v))
        if rc != 0:
            raise EngineError(rc, self.last_error())
        return v.value

    def bench_scan(self, iters=100):
        """Diagnostic: average k_scan device time (us) on the current state."""
        v = C.c_double()
        rc = lib().kb_engine_bench_scan(self.h, iters, C.byref(v))
        if rc < 0:
            raise EngineError(rc, self.last_error())
        return v.value

    # ---- RCCL-driven sharded plan (kb_engine_comm_init / kb_engine_sharded_plan)
    def comm_init(self, n_ranks, rank, uid):
        assert len(uid) == KB_COMM_ID_BYTES
        rc = lib().kb_engine_comm_init(self.h, n_ranks, rank, uid)
        if rc != 0:
            raise EngineError(rc, self.last_error())

    def sharded_plan_raw(self, max_steps):
        """The sharded plan call alone (RCCL all-gather per step, 64 steps per host round
        trip): (change buffer, n, rc); the buffer is reused like plan_raw's."""
        if max_steps > self._cap:
            while self._cap < max_steps:
                self._cap *= 2
            self._buf = (kb_change * self._cap)()
        n = C.c_int64()
        rc = lib().kb_engine_sharded_plan(self.h, max_steps, self._buf, C.byref(n))
        return self._buf, n.value, rc

    def sharded_plan(self, max_steps):
        return self.changes(*self.sharded_plan_raw(max_steps))

    # multi-GPU step phases
    def summary_bytes(self):
        return lib().kb_engine_summary_bytes(self.h)

    def set_stream(self, stream_ptr):
        return lib().kb_engine_set_stream(self.h, C.c_void_p(stream_ptr))

    def step_begin(self, summary_ptr):
        rc = lib().kb_engine_step_begin(self.h, C.c_void_p(summary_ptr))
        if rc < 0:
            raise EngineError(rc, self.last_error())

    # ---- batched sharded steps (no host round trip per step)
    def sharded_reset(self, budget):
        rc = lib().kb_engine_sharded_reset(self.h, budget)
        if rc < 0:
            raise EngineError(rc, self.last_error())

    def sharded_scan(self, summary_ptr):
        rc = lib().kb_engine_sharded_scan(self.h, C.c_void_p(summary_ptr))
        if rc < 0:
            raise EngineError(rc, self.last_error())

    def sharded_resolve(self, gathered_ptr, n_ranks):
        rc = lib().kb_engine_sharded_resolve(self.h, C.c_void_p(gathered_ptr), n_ranks)
        if rc < 0:
            raise EngineError(rc, self.last_error())

    def sharded_collect(self, cap):
        """(status, changes): status "ok" / "retry" (go on), "done" (no change), or raises."""
        buf = (kb_change * max(1, cap))()
        n = C.c_int64()
        rc = lib().kb_engine_sharded_collect(self.h, buf, cap, C.byref(n))
        changes = [_change_dict(buf[i]) for i in range(n.value)]
        if rc < 0:
            raise EngineError(rc, self.last_error(), changes[-1] if changes else None)
        if rc == KB_NOCHANGE:
            return "done", changes[:-1]
        if rc == KB_GROW:
            return "grow", changes                # summary_bytes() grew: new buffers, go on
        return ("retry" if rc == KB_RETRY else "ok"), changes

    def step_finish(self, gathered_ptr, n_ranks):
        """The merged step; None for no change, "retry" when the step must be redone
        (its loads were refolded exactly first); raises EngineError."""
        ch = kb_change()
        rc = lib().kb_engine_step_finish(self.h, C.c_void_p(gathered_ptr), n_ranks, C.byref(ch))
        if rc == KB_NOCHANGE:
            return None
        if rc == KB_RETRY:
            return "retry"
        if rc == KB_GROW:
            return "grow"
        if rc == KB_CHANGE:
            return _change_dict(ch)
        raise EngineError(rc, self.last_error(), _change_dict(ch))

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().kb_engine_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
