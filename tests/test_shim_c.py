"""The C ABI driven from plain C exactly as INTEGRATION.md's cgo shim drives it
(tests/c/shim_test.c: malloc'd arrays only, kb_engine_create once, one
kb_engine_balance per Balance() call -- or the reference's steps table walked on the host,
one kb_engine_step per entry -- with Go aliasing semantics, the reference's error text
from kb_engine_last_error), compared with the oracle's Balance() sequence
(balancer.go:49-65) on the reference fixture test/test.json and on the committed
golden plans."""
import os
import random
import subprocess

import pytest

from oracle import oracle as O

from helpers import default_cfg, golden
from test_gpu_parity_data import random_plist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "kafkabalancer_amd", "lib", "kb_shim_test")
KIND = {1: "replace", 2: "remove", 3: "add", 4: "swap"}


def _cfg_line(cfg):
    br = cfg.get("brokers")
    return " ".join([str(int(bool(cfg.get("allow_leader")))), str(int(bool(cfg.get("rebalance_leaders")))),
                     str(int(cfg.get("min_replicas", 2))), repr(float(cfg.get("min_unbalance", 0.01))),
                     str(int(br is None)), str(len(br or []))] + [str(x) for x in (br or [])])


def shim_input(plist, cfgs, steps, mode=0):
    """cfgs: one config or a list (Balance() call s uses cfgs[s % len(cfgs)])."""
    if isinstance(cfgs, dict):
        cfgs = [cfgs]
    parts = plist["partitions"]
    out = [str(len(parts))]
    for p in parts:
        reps = p.get("replicas") or []
        b = p.get("brokers")
        row = [p["topic"], str(p["partition"]), str(len(reps))] + [str(r) for r in reps]
        row += [repr(float(p.get("weight", 0) or 0)), str(int(p.get("num_replicas", 0) or 0)),
                str(int(p.get("num_consumers", 0) or 0))]
        row += ["-1"] if b is None else [str(len(b))] + [str(x) for x in b]
        out.append(" ".join(row))
    out.append(str(len(cfgs)))
    out += [_cfg_line(c) for c in cfgs]
    out.append("%d %d" % (steps, mode))
    return "\n".join(out) + "\n"


def run_shim(tmp_path, plist, cfgs, steps, mode=0):
    path = tmp_path / "in.txt"
    path.write_text(shim_input(plist, cfgs, steps, mode))
    r = subprocess.run([BIN, str(path)], capture_output=True, text=True, timeout=120)
    lines = r.stdout.splitlines()
    if r.returncode == 0:
        # every engine the shim created was destroyed
        tail = lines.pop().split()
        assert tail[0] == "engines" and tail[1] == tail[2] and int(tail[1]) >= 1, tail
    return r.returncode, lines


def oracle_lines(plist, cfgs, steps):
    if isinstance(cfgs, dict):
        cfgs = [cfgs]
    o = O.OraclePL(plist)
    lines = []
    for s in range(steps):
        r = O.balance(o, cfgs[s % len(cfgs)], O.SEM_GO)
        if r["status"] == 0:
            lines.append("nochange")
            break
        if r["status"] < 0:
            lines.append(("error", r["err"]))
            break
        lines.append("change %d %d %s %d %d %d" % (O.STEP_NAMES.index(r["step"]), r["pidx"], r["kind"],
                                                   r["from_"], r["to"], r["slot"]))
    return lines


def normalize(lines):
    out = []
    for ln in lines:
        f = ln.split(" ", 2)
        if f[0] == "change":
            g = ln.split()
            out.append("change %s %s %s %s %s %s" % (g[1], g[2], KIND[int(g[3])], g[4], g[5], g[6]))
        elif f[0] == "error":
            out.append(("error", f[2]))
        else:
            out.append(ln)
    return out


def test_shim_binary_built_and_linked():
    """CPU check: the shim program links against libkbengine.so and reports a HIP error
    (not a crash) when no GPU is visible."""
    assert os.path.exists(BIN)
    r = subprocess.run(["ldd", BIN], capture_output=True, text=True)
    assert "libkbengine.so" in r.stdout and "not found" not in r.stdout


CASES = ["default", "leader", "rebalance", "brokers6"]


def assert_lines(got, want):
    for a, b in zip(got, want):
        if isinstance(b, tuple) and ": panic" in b[1]:
            assert isinstance(a, tuple) and ": panic" in a[1]
        else:
            assert a == b
    assert len(got) == len(want), (got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["balance", "steps-table"])
@pytest.mark.parametrize("variant", CASES)
def test_shim_matches_oracle_on_test_json(variant, mode, tmp_path):
    pl = golden("test.json")
    cfg = default_cfg()
    if variant == "leader":
        cfg["allow_leader"] = True
    elif variant == "rebalance":
        cfg.update(rebalance_leaders=True, min_unbalance=0.0)
    elif variant == "brokers6":
        cfg["brokers"] = [1, 2, 3, 4, 5, 6]
    rc, lines = run_shim(tmp_path, pl, cfg, 12, mode)
    assert rc == 0, lines
    assert_lines(normalize(lines), oracle_lines(pl, cfg, 12))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["balance", "steps-table"])
def test_shim_matches_golden_go_semantics(mode, tmp_path):
    """Every Go-semantics plan of tests/golden/plans_small.json through the C shim."""
    g = golden("plans_small.json")
    n = 0
    for case in g["cases"]:
        if case["sem"] != "go":
            continue
        rc, lines = run_shim(tmp_path, case["plist"], case["cfg"], case["steps"], mode)
        assert rc == 0, (case["name"], lines)
        got = [ln.split() for ln in lines if ln.startswith("change")]
        want = [[str(O.STEP_NAMES.index(c[0])), str(c[1]), c[2], str(c[3]), str(c[4]), str(c[5])]
                for c in case["changes"]]
        assert [[x[1], x[2], KIND[int(x[3])], x[4], x[5], x[6]] for x in got] == want, case["name"]
        if case["err"] is not None and ": panic" not in case["err"]:
            assert lines[-1].split(" ", 2)[2] == case["err"], case["name"]
        n += 1
    assert n >= 4


ALTERNATING = [
    # (name, configs): Balance() call s runs with configs[s % len(configs)]
    ("leader-toggle", [dict(allow_leader=True, min_unbalance=0.0), dict(allow_leader=False, min_unbalance=0.0)]),
    ("brokers-then-auto", [dict(brokers=[1, 2, 3, 4, 5, 6], min_unbalance=0.0), dict(min_unbalance=0.0)]),
    ("min-unbalance", [dict(min_unbalance=0.0), dict(min_unbalance=0.5), dict(min_unbalance=1e-6, min_replicas=1)]),
    ("rebalance", [dict(rebalance_leaders=True, min_unbalance=0.0), dict(allow_leader=True, min_unbalance=0.0)]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1], ids=["balance", "steps-table"])
@pytest.mark.parametrize("name,cfgs", ALTERNATING, ids=[a[0] for a in ALTERNATING])
def test_shim_alternating_configs(name, cfgs, mode, tmp_path):
    """A caller that passes a different RebalanceConfig on every Balance() call
    (balancer.go:49 takes cfg per call): the shim rebuilds the engine from pl for each new
    config and destroys the old one; the plan equals the oracle's Balance() sequence with
    the same alternation (FillDefaults' Brokers frozen at the first call, Go aliasing)."""
    cfgs = [default_cfg(**c) for c in cfgs]
    for pl in [golden("test.json")] + [random_plist(random.Random(7000 + s), 40, 7, w, "some", True, False)
                                         for s, w in enumerate(["zipf", "uniform"])]:
        rc, lines = run_shim(tmp_path, pl, cfgs, 16, mode)
        assert rc == 0, lines
        assert_lines(normalize(lines), oracle_lines(pl, cfgs, 16))
