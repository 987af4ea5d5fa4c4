"""CPU tests of the native artefacts: the C-ABI library loads and exports every
symbol include/kbengine.h declares (no compute call without a GPU)."""
import ctypes
import os
import re

from kafkabalancer_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "kbengine.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(kb_[a-z_]+)\s*\(", src)))


def test_library_exports_header():
    syms = header_symbols()
    assert "kb_engine_create" in syms and "kb_engine_plan" in syms
    lib = ctypes.CDLL(E.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(E.EXPORTS) == syms


def test_abi_version():
    assert E.lib().kb_abi_version() == 11


def test_library_is_gfx950_code_object():
    with open(E.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_product_does_not_reference_oracle():
    """The product path never imports, links or calls the oracle."""
    pkg = os.path.join(ROOT, "kafkabalancer_amd")
    for dp, _, fns in os.walk(pkg):
        for fn in fns:
            if fn.endswith((".py", ".cpp", ".hip", ".h", ".hpp", "Makefile")):
                with open(os.path.join(dp, fn), errors="ignore") as f:
                    txt = f.read()
                assert "oracle" not in txt.lower().replace("oracle_free", ""), os.path.join(dp, fn)


def test_broker_universe_limit():
    """Up to MAXB_G = 16384 distinct broker ids (past 4096 the kernels read the broker tables
    from memory); one more is an explicit KB_ERR_UNSUPPORTED, checked before any device call."""
    import pytest
    from kafkabalancer_amd import synth
    cl = synth.make_cluster(10, 40, 3, "int", seed=1)
    cfg = {"allow_leader": False, "rebalance_leaders": False, "min_replicas": 2, "min_unbalance": 0.0,
           "brokers": list(range(1, 16386))}
    with pytest.raises(E.EngineError) as ei:
        E.Engine(cl, cfg)
    assert ei.value.code == -3 and "16384 distinct brokers" in str(ei.value)   # KB_ERR_UNSUPPORTED


def test_diagnostic_switches_need_the_opt_in():
    """The library reads its KB_* A/B and diagnostic switches only after kb_set_diagnostics(1)
    (a drop-in host never calls it): loaded without KB_DIAGNOSTICS the opt-in is off, with it
    the Python binding turns it on."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from kafkabalancer_amd import engine as E; "
            "print(E.lib().kb_diagnostics_enabled())" % root)
    for val, want in ((None, "0"), ("1", "1")):
        env = dict(os.environ, KB_FUSE="0")
        env.pop("KB_DIAGNOSTICS", None)
        if val:
            env["KB_DIAGNOSTICS"] = val
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip().splitlines()[-1] == want, r.stdout
