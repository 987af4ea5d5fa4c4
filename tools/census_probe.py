"""Diagnostic (c3nl census): per step of a plan, the census bound ub, eps and the step's
score (cu - su), to see how wide the census window is against the scores it separates."""
import json
import os

import numpy as np
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3nl"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    cl, cfg, _ = synth.config(wl)
    eng = E.Engine(cl, cfg, device=0)
    for k in range(n):
        before = eng.ctl_scalars()
        ch, err = eng.plan(1)
        assert err is None and ch, err
        c = ch[0]
        rec = eng.debug_records()
        b1 = rec["best"][:, 1]
        v1 = b1["s"] >= 0
        parts = (b1["iter"][v1] >> 21).astype(np.int64)
        rinfo = {"recs": int(len(rec)), "best1_valid": int(v1.sum()), "best1_distinct_parts": int(len(set(parts.tolist()))),
                 "best1_moved_part": int((parts == c["pidx"]).sum()),
                 "dmin1_min": float(rec["dmin"][:, 1].min()), "nkeys_sum": int(rec["nkeys"].sum()),
                 "flags_ovf": int((rec["flags"] & 1).sum())}
        print(json.dumps({"rec": rinfo,"k": k, "pidx": c["pidx"], "d": c["cu"] - c["su"], "su": c["su"], "exact": c["exact"],
                          "ub1": before["ub1"], "ub0": before["ub0"], "eps": before["eps"], "U0": before["U0"],
                          "V": before["V"], "avg": before["avg"], "rlo": before["rlo"], "rhi": before["rhi"]}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
