"""Diagnostic: the scan workgroups' timeline of one steady-state k_pair launch.

Runs WL (default c3) for N steps with KB_WGT set, so the engine records per scan workgroup
{start, scored (all waves past the census), record written} on the 100 MHz device clock and
appends them to a file when it is destroyed; prints the distribution relative to the first
start.   python tools/wg_timeline.py [WL] [N]   (GPU)"""
import json
import os
import sys

import numpy as np
os.environ.setdefault("KB_DIAGNOSTICS", "1")   # (the engine reads its KB_* switches only with this opt-in)

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
    t6 = np.array(x["wg"], dtype=np.int64).reshape(-1, 6)
    t6 = t6[t6[:, 0] > 0]
    t = t6[:, :3]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0
    q = lambda v: [round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)]
    out = {"workload": wl, "steps": len(ch), "wgs": int(len(t)),
           "start_us_pct_0_10_50_90_100": q(us[:, 0]),
           "scored_us": q(us[:, 1]), "end_us": q(us[:, 2]),
           "dur_start_to_scored_us": q(us[:, 1] - us[:, 0]),
           "dur_scored_to_end_us": q(us[:, 2] - us[:, 1])}
    idx = np.nonzero(np.array(x["wg"], dtype=np.int64).reshape(-1, 6)[:, 0] > 0)[0]
    slow = np.argsort(-(us[:, 1] - us[:, 0]))[:6]
    out["slowest"] = [[int(idx[i]), round(float(us[i, 0]), 2), round(float(us[i, 1]), 2), round(float(us[i, 2]), 2),
                       int(t6[i, 3]), int(t6[i, 4]), int(t6[i, 5])] for i in slow]
    out["slowest_def"] = "[wg, start, scored, end (us), census shader clocks summed over its waves, census waves, walk clocks]"
    out["census_wgs"] = int((t6[:, 4] > 0).sum())
    late = np.argsort(-us[:, 2])[:6]
    out["latest_end"] = [[int(idx[i]), round(float(us[i, 0]), 2), round(float(us[i, 1]), 2), round(float(us[i, 2]), 2)] for i in late]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
