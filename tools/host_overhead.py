"""Per-call host overhead of kb_engine_plan at c3: the driver's bench
line times plan_raw(20) between two torch.cuda.synchronize() calls, so everything outside
the device's own 20 steps -- the control-block reset, the batch-end transfer, the wait --
is charged to ms_per_step.  Each variant gets its own engine (the switches are read at
create): KB_XFER 0 (hipMemcpyAsync, round 4), 1 (k_xfer + stream sync), 2 (k_xfer + host
poll, the default), and the two-launch pair (KB_FUSE=0).  Prints one JSON line per
variant: wall and device us per call, their difference per step, and the host phases
(kb_engine_host_timings)."""
import json
import os
import sys
import time
os.environ.setdefault("KB_DIAGNOSTICS", "1")   # (the engine reads its KB_* switches only with this opt-in)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cl, cfg, _ = synth.config(wl)
    variants = [("xfer2", {"KB_XFER": "2"}), ("xfer1", {"KB_XFER": "1"}), ("xfer0", {"KB_XFER": "0"}),
                ("xfer0_nofuse", {"KB_XFER": "0", "KB_FUSE": "0"}), ("xfer2_nofuse", {"KB_XFER": "2", "KB_FUSE": "0"})]
    for name, env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            eng = E.Engine(cl, cfg, device=0)
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        _, err = eng.plan(20)
        assert err is None, err
        for steps in (1, 20, 200):
            walls, devs = [], []
            eng.set_timing(False)          # (resets the host phase sums)
            for _ in range(20 if steps < 200 else 5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                buf, n, rc = eng.plan_raw(steps)
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t0)
                devs.append(eng.stats()["device_ms"] / 1e3)
                assert rc >= 0 and n == steps, (rc, n)
            walls.sort()
            devs.sort()
            w = walls[len(walls) // 2]
            d = devs[len(devs) // 2]
            ht = eng.host_timings()
            calls = max(ht["calls"], 1)
            print(json.dumps({"variant": name, "workload": wl, "steps": steps, "fused": eng.stats()["fused_pairs"],
                              "wall_us_median": 1e6 * w, "device_us_median": 1e6 * d,
                              "wall_minus_device_us_per_step": 1e6 * (w - d) / steps,
                              "ms_per_step": 1e3 * w / steps,
                              "host_us_per_call": {k: v / calls for k, v in ht.items() if k != "calls"}}),
                  flush=True)
        eng.close()


if __name__ == "__main__":
    main()
