"""ctypes binding of libkbcpu.so (tools/cpu_engine/kb_cpu_engine.cpp), the OpenMP
CPU restatement of the engine's algorithm: MEASUREMENT INFRASTRUCTURE (bench.py's
cpu_baseline leg, tests/test_cpu_engine.py); never part of the product."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "kafkabalancer_amd", "lib", "libkbcpu.so")
STEPS = {3: "RemoveExtraReplicas", 4: "AddMissingReplicas", 5: "MoveDisallowedReplicas",
         7: "MoveLeaders", 8: "MoveNonLeaders"}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.abspath(__file__))], check=True)
        L = C.CDLL(LIB)
        P = C.POINTER(C.c_int64)
        L.cpu_engine_create.restype = C.c_void_p
        L.cpu_engine_create.argtypes = [C.c_int64, P, P, C.POINTER(C.c_double), P, P, C.c_int64, P, P, P, P,
                                        C.c_int64, C.c_int, C.c_int, C.c_int64, C.c_double, C.c_int]
        L.cpu_engine_step.argtypes = [C.c_void_p, P, C.POINTER(C.c_double)]
        L.cpu_engine_step.restype = C.c_int
        L.cpu_engine_candidates.argtypes = [C.c_void_p]
        L.cpu_engine_candidates.restype = C.c_int64
        L.cpu_engine_destroy.argtypes = [C.c_void_p]
        _lib = L
    return _lib


class CpuEngine:
    """cl: kafkabalancer_amd.engine.ClusterSoA; cfg: the reference config dict."""

    def __init__(self, cl, cfg, threads=0):
        p64 = C.POINTER(C.c_int64)
        w = np.where(cl.weight == 0, 1.0, cl.weight) if cl.weight[0] == 0 else cl.weight.copy()
        lens = np.diff(cl.replica_off)
        nr = np.where(cl.num_replicas == 0, lens, cl.num_replicas)
        br = cfg.get("brokers")
        self._keep = [np.ascontiguousarray(x) for x in (cl.replica_ids, cl.replica_off, w, nr, cl.num_consumers,
                                                          cl.set_ids, cl.set_off, cl.set_idx,
                                                          np.array(br if br else [0], np.int64))]
        k = self._keep
        self.h = lib().cpu_engine_create(cl.n, k[0].ctypes.data_as(p64), k[1].ctypes.data_as(p64),
                                         k[2].ctypes.data_as(C.POINTER(C.c_double)), k[3].ctypes.data_as(p64),
                                         k[4].ctypes.data_as(p64), len(cl.set_off) - 1, k[5].ctypes.data_as(p64),
                                         k[6].ctypes.data_as(p64), k[7].ctypes.data_as(p64),
                                         k[8].ctypes.data_as(p64), len(br or []), int(br is None),
                                         int(bool(cfg.get("allow_leader"))), int(cfg.get("min_replicas", 2)),
                                         float(cfg.get("min_unbalance", 0.01)), int(threads))
        if not self.h:
            raise ValueError("cluster outside the CPU engine's scope (empty replica lists or > 64 slots)")

    def step(self):
        oi = (C.c_int64 * 5)()
        od = (C.c_double * 2)()
        rc = lib().cpu_engine_step(self.h, oi, od)
        if rc < 0:
            raise RuntimeError("%s: the reference errors here" % STEPS.get(oi[0], "step"))
        if rc != 1:
            return None
        return {"step": STEPS[oi[0]], "pidx": oi[1], "slot": oi[2], "from_": oi[3], "to": oi[4],
                "su": od[0], "cu": od[1]}

    def candidates(self):
        return lib().cpu_engine_candidates(self.h)

    def close(self):
        if self.h:
            lib().cpu_engine_destroy(self.h)
            self.h = None
