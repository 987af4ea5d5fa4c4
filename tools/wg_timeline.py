"""Diagnostic: the scan workgroups' timeline of one steady-state k_pair launch.

Runs WL (default c3) for N steps with KB_WGT set, so the engine records per scan workgroup
{start, scored (all waves past the census), record written} on the 100 MHz device clock and
appends them to a file when it is destroyed; prints the distribution relative to the first
start.   python tools/wg_timeline.py [WL] [N]   (GPU)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    path = os.path.join(ROOT, "gpurun_out", "wgt_%s.jsonl" % wl)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        os.remove(path)
    os.environ["KB_WGT"] = path
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    cl, cfg, _ = synth.config(wl)
    eng = E.Engine(cl, cfg, device=0, time_kernels=False)
    ch, err = eng.plan(n)
    assert err is None, err
    eng.close()
    x = [json.loads(ln) for ln in open(path)][-1]
    t = np.array(x["wg"], dtype=np.int64).reshape(-1, 3)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0
    q = lambda v: [round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)]
    out = {"workload": wl, "steps": len(ch), "wgs": int(len(t)),
           "start_us_pct_0_10_50_90_100": q(us[:, 0]),
           "scored_us": q(us[:, 1]), "end_us": q(us[:, 2]),
           "dur_start_to_scored_us": q(us[:, 1] - us[:, 0]),
           "dur_scored_to_end_us": q(us[:, 2] - us[:, 1])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
