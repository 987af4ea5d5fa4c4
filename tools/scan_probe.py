"""Diagnostic: isolated k_scan timing on the c3 state under the KB_DEBUG_SCAN knobs.
With KB_ENGINE_LIB pointing at libkbengine_stamps.so it also prints the census
event counters (walks, walk iterations, emits, spills) per scan launch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kafkabalancer_amd import engine as E  # noqa: E402
from kafkabalancer_amd import synth  # noqa: E402

cl, cfg, _ = synth.config(sys.argv[1] if len(sys.argv) > 1 else "c3")
eng = E.Engine(cl, cfg)
eng.plan(int(os.environ.get("KB_PROBE_STEPS", "5")))
st0 = eng.stamps()
iters = 200
us = eng.bench_scan(iters)
st1 = eng.stamps()
out = {"dbg": os.environ.get("KB_DEBUG_SCAN", "0"), "nscan": eng.stats()["scan_workgroups"], "scan_us": us}
if "stamps" in os.environ.get("KB_ENGINE_LIB", ""):
    d = [(b - a) / (iters + 1) for a, b in zip(st0, st1)]
    out["per_scan"] = {"beyond_iters": d[27], "spills": d[30], "walks": d[29], "walk_iters": d[28], "emits": d[31]}
print(json.dumps(out))
