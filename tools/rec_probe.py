"""Diagnostic: the last scan's records after N steps of WL -- which records hold near-tie keys
(nkeys / nkk per kind), their minima against the step's, and the engine's spill count.
python tools/rec_probe.py [WL] [N] [rec ...]   (GPU)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    watch = [int(v) for v in sys.argv[3:]]
    cl, cfg, _ = synth.config(wl)
    eng = E.Engine(cl, cfg, device=0, time_kernels=False)
    ch, err = eng.plan(n)
    assert err is None, err
    rec = eng.debug_records()
    sc = eng.ctl_scalars()
    g = rec["dmin"].min(axis=0)
    nk = rec["nkeys"].astype(np.int64)
    out = {"workload": wl, "steps": len(ch), "records": int(len(rec)), "eps": sc["eps"], "g": g.tolist(),
           "records_with_keys": int((nk > 0).sum()), "keys_total": int(nk.sum()),
           "nkk_total": [int(rec["nkk"][:, 0].sum()), int(rec["nkk"][:, 1].sum())],
           "top_nkk": sorted([[int(i), int(rec["nkk"][i, 0]), int(rec["nkk"][i, 1]), int(nk[i])]
                              for i in range(len(rec))], key=lambda v: -(v[1] + v[2]))[:8],
           "stats": {k: v for k, v in eng.stats().items() if k in ("contenders", "candidates", "steps")},
           "last_changes": [c for c in ch[-2:]]}
    for i in watch:
        out["rec%d" % i] = {"dmin": rec["dmin"][i].tolist(), "nkeys": int(nk[i]), "nkk": rec["nkk"][i].tolist(),
                            "d_minus_g_over_eps": ((rec["dmin"][i] - g) / sc["eps"]).tolist()}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
