"""The native host code under AddressSanitizer + UBSan (host code only:
no GPU is touched, and the device kernels are never built with a sanitizer).

* `tests/c/host_fuzz.cpp` links the host side (kafkabalancer_amd/host: the JSON and
  `--describe` codecs, codecs.go:15-93, and the CLI, kafkabalancer.go:72-242) built
  with -fsanitize=address,undefined and drives it with mutated documents and argument
  vectors; the one-pass JSON decoder must also agree with the DOM decoder on every
  mutated document.
* The engine's host half (`kafkabalancer_amd/csrc/engine.cpp`: the marshalling and the
  Validate*/FillDefaults checks of kb_engine_create, balancer.go:34-44, steps.go:7-66)
  built with `-Xarch_host -fsanitize=address,undefined`, loaded by a Python
  subprocess with libasan preloaded, creating engines from random and malformed
  clusters; without a GPU every create ends at hipSetDevice, after the host work.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "kafkabalancer_amd", "lib")
HOST = os.path.join(ROOT, "kafkabalancer_amd", "host")
CSRC = os.path.join(ROOT, "kafkabalancer_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]


def _asan_runtime():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) else None


def _seeds(tmp_path):
    sys.path.insert(0, ROOT)
    import json
    from kafkabalancer_amd import synth
    cl = synth.make_cluster(40, 12, 3, "zipf", nsets=4, set_size=6, seed=9, with_names=True)
    js = tmp_path / "seed.json"
    js.write_text(json.dumps(synth.to_plist(cl)))
    lines = ["Topic:t00000\tPartitionCount:30\tReplicationFactor:3\tConfigs:"]
    for i in range(30):
        r = [1 + i % 5, 1 + (i + 1) % 5, 1 + (i + 2) % 5]
        lines.append("\tTopic: t%05d\tPartition: %d\tLeader: %d\tReplicas: %s\tIsr: %s"
                     % (i // 10, i % 10, r[0], ",".join(map(str, r)), ",".join(map(str, r[:2]))))
    tx = tmp_path / "seed.txt"
    tx.write_text("\n".join(lines) + "\n")
    return str(js), str(tx)


def test_host_codecs_and_cli_under_asan_ubsan(tmp_path):
    if not os.path.exists(os.path.join(LIB, "libkbengine.so")):
        pytest.skip("libkbengine.so not built")
    exe = str(tmp_path / "host_fuzz")
    src = [os.path.join(ROOT, "tests", "c", "host_fuzz.cpp")] + \
          [os.path.join(HOST, f) for f in ("codecs.cpp", "cli.cpp", "balancer.cpp")]
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-ffp-contract=off"] + SAN +
                   ["-o", exe] + src + ["-L" + LIB, "-lkbengine", "-Wl,-rpath," + LIB], check=True)
    js, tx = _seeds(tmp_path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, js, tx, "20000"], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0 and "host-fuzz-ok 20000" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


ENGINE_SCRIPT = r'''
import random, sys
import numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, %(tests)r)
from kafkabalancer_amd import engine as E
E.LIB_PATH = %(lib)r
from test_gpu_parity_data import random_plist
ok = 0
for seed in range(300):
    rng = random.Random(seed)
    pl = random_plist(rng, rng.choice([0, 1, 10, 40, 120]), rng.choice([1, 3, 5, 9, 70]),
                      rng.choice(["uniform", "int", "zipf"]), rng.choice(["none", "some", "all"]),
                      rng.random() < 0.5, rng.random() < 0.3)
    for p in pl["partitions"]:
        r = rng.random()
        if r < 0.03:
            p["replicas"] = (p.get("replicas") or []) * 2             # duplicates / too many slots
        elif r < 0.05:
            p["weight"] = -1.0
        elif r < 0.07:
            p["num_consumers"] = rng.choice([-5, 1 << 31])
        elif r < 0.09:
            p["weight"] = float("inf")
        elif r < 0.11:
            p["brokers"] = []
    cfg = {"allow_leader": rng.random() < 0.5, "min_unbalance": 0.0,
           "brokers": None if rng.random() < 0.5 else list(range(1, rng.choice([2, 12, 5000])))}
    shard = None if rng.random() < 0.8 else (rng.choice([0, 7, 1024]), rng.choice([0, 5, 40]))
    try:
        E.Engine(pl, cfg, shard=shard).close()
    except E.EngineError as ex:
        ok += 1
print("engine-asan-ok", ok)
'''


def test_engine_host_half_under_asan_ubsan(tmp_path):
    asan = _asan_runtime()
    if not asan:
        pytest.skip("libasan not available")
    lib = str(tmp_path / "libkbengine_asan.so")
    hip = "/opt/rocm/bin/hipcc"
    kobj = str(tmp_path / "kernels.o")
    eobj = str(tmp_path / "engine.o")
    common = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off"]
    # device code unchanged and unsanitized; the host half with the sanitizers
    subprocess.run([hip] + common + ["-c", os.path.join(CSRC, "kernels.hip"), "-o", kobj], check=True,
                   capture_output=True)
    host_san = []
    # (clang's -fsanitize=function check of indirect calls -- the RCCL entry points the
    # engine binds with dlsym -- needs a handler gcc's libubsan does not have)
    for f in SAN + ["-fno-sanitize=function"]:
        host_san += ["-Xarch_host", f]
    subprocess.run([hip] + common + host_san + ["-x", "hip", "-c", os.path.join(CSRC, "engine.cpp"), "-o", eobj],
                   check=True, capture_output=True)
    # (the host linker: the device code objects ride along in kernels.o's bundle)
    subprocess.run(["g++", "-shared"] + SAN + ["-o", lib, kobj, eobj, "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True, capture_output=True)
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    pre = asan + (":" + ubsan if os.path.isabs(ubsan) else "")
    env = dict(os.environ, LD_PRELOAD=pre, PYTHONMALLOC="malloc", ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               HIP_VISIBLE_DEVICES="")
    code = ENGINE_SCRIPT % {"root": ROOT, "tests": os.path.join(ROOT, "tests"), "lib": lib}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0 and "engine-asan-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
