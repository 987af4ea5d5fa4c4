"""Summarise a tools/gpu_r05.sh output directory: python tools/show_r05.py gpurun_out/<tag>"""
import json
import os
import sys


def last_json(path):
    try:
        with open(path) as f:
            lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except OSError:
        return None


def main():
    d = sys.argv[1]
    p = os.path.join(d, "pytest_gpu.log")
    if os.path.exists(p):
        with open(p) as f:
            print("pytest:", f.read().strip().splitlines()[-1])
    pr = os.path.join(d, "probe.jsonl")
    if os.path.exists(pr):
        for ln in open(pr):
            x = json.loads(ln)
            print("probe", x["k"], x["pidx"], "d=%.3e ub0=%.3e ub1=%.3e" % (x["d"], x["ub0"], x["ub1"]), x.get("rec"))
    for wl in ("c2", "c3", "c3_acq", "c3b", "c3nl", "c5"):
        x = last_json(os.path.join(d, wl + ".json"))
        if not x:
            continue
        r = x["roofline"]
        print(wl, "ms/step %.4f dev %.4f launch %.1f us frac %.3f scan %.1f" % (
            x["ms_per_step"], x["config"]["device_ms_per_step"], r["avg_launch_us"], r["frac"], r.get("scan_phase_us") or 0),
            {k: round(v, 1) for k, v in x["kernels_us_per_launch"].items()}, x["engine_events"])
    for wl in ("c2", "c3", "c3nl", "c5"):
        x = last_json(os.path.join(d, wl + "_stamps.json"))
        if x:
            st = {k: round(v, 2) for k, v in x["stamps_us_per_step"].items() if v >= 0.3}
            print(wl, "stamps k_step %.1f us" % x["k_step_us"], st)
    for f in ("sharded", "sharded_nofuse"):
        x = last_json(os.path.join(d, f + ".json"))
        if x:
            print(f, {k: x[k] for k in ("ms_per_step_sharded", "ms_per_step_plain", "ratio", "plans_equal")})


if __name__ == "__main__":
    main()
