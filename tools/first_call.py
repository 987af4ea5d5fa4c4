"""The driver's bench sequence (bench.py main: create, plan(W) warm-up, one timed plan_raw(K)
between torch.cuda.synchronize() calls), then the same timed call repeated: is the first
timed call's wall - device larger than the later ones', and in which host phase?"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    K, W = int(sys.argv[1]), int(sys.argv[2])
    cl, cfg, desc = synth.config("c3")
    eng = E.Engine(cl, cfg, device=0, time_kernels=False)
    _, err = eng.plan(W)
    assert err is None
    prev = eng.host_timings()
    for i in range(6):
        eng.stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        raw = eng.plan_raw(K)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        dev = eng.stats()["device_ms"] / 1e3
        print(json.dumps({"call": i, "K": K, "W": W, "wall_us": 1e6 * wall, "device_us": 1e6 * dev,
                          "gap_us_per_step": 1e6 * (wall - dev) / K, "ms_per_step": 1e3 * wall / K,
                          "host": {k: v - prev[k] for k, v in eng.host_timings().items()}}), flush=True)
        prev = eng.host_timings()
    eng.close()


if __name__ == "__main__":
    main()
