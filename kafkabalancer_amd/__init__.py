"""kafkabalancer_amd: MI355X-native move-search engine for kafkabalancer's Balance() pipeline.

The hot path (steps.go move search + Remove/Add/Disallowed predicates) runs as
HIP kernels for gfx950 behind the C ABI in include/kbengine.h
(kafkabalancer_amd/lib/libkbengine.so).  Python modules here are thin hosts:
  engine.py   ctypes binding of the C ABI (no CPU fallback)
  api.py      mirror of the reference Go API (PartitionList, Balance, ...)
  synth.py    BASELINE.json synthetic workloads
"""
__all__ = ["engine", "synth"]
