"""The C oracle under AddressSanitizer + UBSan (host code only), in a subprocess with
libasan preloaded: multi-step plans over explicit -broker-ids lists, Go aliasing
semantics, removes/adds, the threaded move() and the run() writer.  Regression pin for
the oracle once sharing the caller's cfg.Brokers array across Balance() calls."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import random, sys
sys.path.insert(0, %(root)r); sys.path.insert(0, %(tests)r)
from oracle import oracle as O
O._LIB_PATH = %(lib)r
from test_gpu_parity_data import random_plist
for seed in range(30):
    rng = random.Random(seed)
    pl = random_plist(rng, rng.choice([10, 40, 120]), rng.choice([3, 5, 9]),
                      rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                      rng.random() < 0.5, rng.random() < 0.3)
    cfg = dict(O.default_cfg(), allow_leader=rng.random() < 0.5, rebalance_leaders=rng.random() < 0.3,
               min_unbalance=rng.choice([0.0, 0.01]), min_replicas=rng.choice([1, 2, 3]))
    if seed %% 2:
        cfg["brokers"] = list(range(1, 12))
    O.set_threads(1 + seed %% 3)
    for sem in (O.SEM_APPLIED, O.SEM_GO):
        o = O.OraclePL(pl)
        for _ in range(25):
            if O.balance(o, cfg, sem)["status"] != 1:
                break
    O.run_plan(O.OraclePL(pl), cfg, max_reassign=5, complete_partition=False, full_output=True, unique=True)
print("asan-ok")
'''


def test_oracle_clean_under_asan(tmp_path):
    lib = str(tmp_path / "libkboracle_asan.so")
    src = os.path.join(ROOT, "oracle", "kb_oracle.c")
    subprocess.run(["gcc", "-O1", "-g", "-fPIC", "-ffp-contract=off", "-fopenmp",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-shared",
                    "-o", lib, src, "-lm"], check=True)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan):
        pytest.skip("libasan not available")
    env = dict(os.environ, LD_PRELOAD=asan, PYTHONMALLOC="malloc", ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    code = SCRIPT % {"root": ROOT, "tests": os.path.join(ROOT, "tests"), "lib": lib}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "asan-ok" in r.stdout, r.stderr[-4000:]
