"""Diagnostic: per-phase device-clock times of the eager workgroups at c5 (a build with
ctl.stamps[16..23,26] instrumentation in eager_edit_refold, KB_ENGINE_LIB=...diag2.so)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from kafkabalancer_amd import engine as E  # noqa: E402
from kafkabalancer_amd import synth  # noqa: E402

torch.cuda.set_device(0)
cl, cfg, _ = synth.config(sys.argv[1] if len(sys.argv) > 1 else "c5")
eng = E.Engine(cl, cfg, device=0)
eng.plan(20)
st0 = eng.stamps()
t = time.perf_counter()
eng.plan(int(sys.argv[2]) if len(sys.argv) > 2 else 100)
st = eng.stamps()
d = [int(st[i]) - int(st0[i]) for i in range(32)]
n = max(d[21], 1)
print(json.dumps({"eager_one_pass": d[21], "entries_us": d[16] / n / 100.0, "gather_us": d[17] / n / 100.0,
                  "chain_us": d[18] / n / 100.0, "chain_len": d[19] / n, "list_len": d[20] / n,
                  "op_mean": d[22] / n, "pre_us": d[23] / max(d[26], 1) / 100.0, "one": d[26]}))
