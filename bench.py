"""Benchmark: candidate moves scored/sec + ms per reassignment step on MI355X.

Workload (N=1): BASELINE.json configs[2] -- synthetic 1M partitions x 1000
brokers, RF3, Zipf weights, 256 allowed-broker sets of 64, -allow-leader,
-min-unbalance 0 (the metric's "1M partitions x 1k brokers").  A step is one
Balance() call (balancer.go:49-65) executed device-resident by
kb_engine_plan; `value` counts the candidates the reference would score
(SURVEY.md 8d metric 1) over the timed steps.

Multi-GPU (torchrun): weak scaling, every rank holds the full cluster state
(N x 1M partitions, replicated) and scans its own 1M-partition shard; one
all-gather of a fixed-size summary per step combines the ranks.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def cpu_baseline(cl, cfg, seconds=12.0):
    """The oracle (C restatement of steps.go move(), single thread) on a bounded
    sample: the first k partitions of the same cluster, leader step (the step
    the reference runs first with -allow-leader)."""
    from oracle import oracle as O
    P = cl.n
    blob = b"t"
    toff = np.zeros(P + 1, np.int64)
    toff[1:] = 1
    opl = O.OraclePL.from_soa(blob * 1, np.zeros(P + 1, np.int64), np.arange(P, dtype=np.int64),
                              cl.replica_ids, cl.replica_off, np.where(cl.weight == 0, 1.0, cl.weight),
                              np.where(cl.num_replicas == 0, 3, cl.num_replicas),
                              cl.set_ids, cl.set_off, cl.set_idx, cl.num_consumers)
    k = 16
    while True:
        t0 = time.perf_counter()
        n, _ = O.move_sample(opl, cfg, True, k)
        dt = time.perf_counter() - t0
        if dt > seconds / 8 or k >= P:
            break
        k = min(P, int(k * max(2.0, (seconds / 8) / max(dt, 1e-4))))
    k2 = min(P, int(k * seconds / max(dt, 1e-6)))
    if k2 > k:
        t0 = time.perf_counter()
        n, _ = O.move_sample(opl, cfg, True, k2)
        dt = time.perf_counter() - t0
        k = k2
    return {"value": n / dt, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": "oracle move(leaders) over the first %d of %d partitions: %d candidates in %.1f s "
                      "(reference Go not buildable: no Go toolchain)" % (k, P, n, dt)}


def pmc_traffic(kernel):
    """HBM-side bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_bench.sh)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f)[kernel]["traffic_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: load the -DKB_STAMPS build and print per-phase times (not a bench line)")
    args = ap.parse_args()
    if args.stamps:
        os.environ["KB_ENGINE_LIB"] = os.path.join(ROOT, "kafkabalancer_amd", "lib", "libkbengine_stamps.so")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        from kafkabalancer_amd import dist
        return dist.bench_main(args, world, rank, local)

    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    cl, cfg, desc = synth.config(args.workload, scale=args.scale)
    eng = E.Engine(cl, cfg, device=0, time_kernels=False)
    if args.warmup:
        _, err = eng.plan(args.warmup)
        assert err is None, err
    st0 = eng.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    changes, err = eng.plan(args.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    assert err is None, err
    st1 = eng.stats()
    steps = len(changes) + (0 if len(changes) == args.steps else 1)
    cand = st1["candidates"] - st0["candidates"]
    dev_s = st1["device_ms"] / 1e3
    # per-kernel durations, outside the headline timing above (instrumentation
    # between the launches adds its own gaps):
    #  * device clock: every scan workgroup stamps its start/end, k_step folds the
    #    interval (earliest start .. latest end) -- a second stretch of the same plan;
    #  * HIP events on the engine's stream around 200 back-to-back k_scan launches
    #    on the plan's final state: dispatch-inclusive, the interval rocprofv3
    #    reports.  `achieved` uses this (the conservative) one.
    eng.set_timing(True)
    kt_steps = min(args.steps, 200)
    _, err = eng.plan(kt_steps)
    assert err is None, err
    tk = eng.timings()
    scan_ms, scan_n = tk["scan"]
    scan_clock_us = 1e3 * scan_ms / max(scan_n, 1)
    eng.set_timing(False)
    scan_avg_us = eng.bench_scan(200)
    bytes_scan = st1["scan_bytes"]
    achieved = bytes_scan / (scan_avg_us * 1e-6) / 1e9
    out = {
        "metric": "candidate moves scored/sec (+ ms per reassignment step)",
        "value": cand / wall,
        "unit": "candidates/s",
        "n_gpus": 1,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * wall / max(steps, 1),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (numpy PCG64 seed 0x5EED0003), Zipf weights r^-1.1",
        "config": dict(desc, parallelism="single-gpu", device_ms_per_step=1e3 * dev_s / max(steps, 1)),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("k_scan"),
                     "kernel": "k_scan", "bytes_per_launch": bytes_scan,
                     "avg_launch_us": scan_avg_us,
                     "timing": "HIP events on the engine stream around 200 back-to-back k_scan launches "
                               "(dispatch-inclusive, as rocprofv3 kernel-trace)",
                     "avg_launch_us_device_clock": scan_clock_us,
                     "frac_device_clock": bytes_scan / (scan_clock_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                     "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch)"},
        "kernels_us_per_step": {k: 1e3 * v[0] / max(v[1], 1) for k, v in tk.items()},
        "kernel_timing_steps": kt_steps,
        "engine_events": {k: st1[k] - st0[k] for k in ("retries", "refreshes", "exact_halts", "exact_folds")},
    }
    if args.stamps:
        st = eng.stamps()
        n = max(1, eng.stats()["steps"])       # every step since the engine was created
        names = ["prep.S+r+ubloop", "step.loads", "res.reduce", "res.pred", "res.move", "res.apply(tail)", "prep.sort", None,
                 "prep.blm+cert", "prep.reduce+eps", "prep.sets", "res.move->apply", "loads.bro+ctl", "loads.rec_reduce", "loads.keys", None, "sets.mark", "eps.sync1", "eps.wave0red", "sets.list", "sets.build", "keys.pre", "keys.insert"]
        counts = {"waves_scored": 7, "waves_gated_in": 15, "emits": 31, "spills": 30, "walks": 29, "walk_steps": 28, "walk_global": 27}
        print(json.dumps({"k_step_clock_mhz": 100.0 * st[25] / max(st[24], 1),
                          "k_step_us": st[24] / 100.0 / n,
                          "stamps_us_per_step": {k: st[i] / 100.0 / n for i, k in enumerate(names) if k},
                          "counts_per_step": {k: st[i] / n for k, i in counts.items()},
                          "stats": eng.stats()}))
        return
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cl, cfg, args.cpu_seconds)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
