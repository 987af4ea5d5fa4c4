"""kafkabalancer_amd: MI355X-native move-search engine for kafkabalancer's Balance() pipeline.

The hot path (steps.go move search + Remove/Add/Disallowed predicates) runs as
HIP kernels for gfx950 behind the C ABI in include/kbengine.h
(kafkabalancer_amd/lib/libkbengine.so).  Python modules here are thin hosts:
  engine.py   ctypes binding of the C ABI (no CPU fallback)
  dist.py     multi-GPU plan driver (partition shards, one all-gather per step)
  cli.py      the C++ CLI (host/, the reference's run() and codecs) from Python
  synth.py    BASELINE.json synthetic workloads
The reference's Go API surface (PartitionList, Balance, the steps table) is mirrored by
the C++ host library in host/ and, from Go, by the cgo shim in INTEGRATION.md.
"""
__all__ = ["engine", "synth"]
