"""Diagnostic: c5 (10M partitions x 4096 brokers) step by step: wall time per
Balance() call and the engine's event counters (retries, refreshes, folds)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kafkabalancer_amd import engine as E  # noqa: E402
from kafkabalancer_amd import synth  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cl, cfg, _ = synth.config("c5", scale=scale)
eng = E.Engine(cl, cfg)
for i in range(steps):
    t0 = time.perf_counter()
    ch, err = eng.plan(1)
    dt = time.perf_counter() - t0
    st = eng.stats()
    print(json.dumps({"i": i, "ms": 1e3 * dt, "err": str(err) if err else None,
                      "pidx": ch[0]["pidx"] if ch else None,
                      **{k: st[k] for k in ("contenders", "exact_folds", "refreshes", "exact_halts", "retries")}}),
          flush=True)
    if err:
        break
t0 = time.perf_counter()
ch, err = eng.plan(20)
print(json.dumps({"plan20_ms": 1e3 * (time.perf_counter() - t0), "n": len(ch), "err": str(err) if err else None,
                  "retries": eng.stats()["retries"]}), flush=True)
