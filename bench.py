"""Benchmark: candidate moves scored/sec + ms per reassignment step on MI355X.

Workload (N=1): BASELINE.json configs[2] -- synthetic 1M partitions x 1000
brokers, RF3, Zipf weights, 256 allowed-broker sets of 64, -allow-leader,
-min-unbalance 0 (the metric's "1M partitions x 1k brokers").  A step is one
Balance() call (balancer.go:49-65) executed device-resident by kb_engine_plan;
`value` counts the candidates the reference would score (SURVEY.md 8d metric 1)
over the timed steps, per wall second.

Roofline: the dominant kernel is the launch that streams the partitions --
k_pair (the scan's grid and the step workgroup in one launch per step) where the engine
fuses the pair, else k_scan; `achieved` = SURVEY 8(d)'s algorithmic bytes of a step (26.0 MB
at c3; the engine's own 18-B-per-partition layout is a side figure) / that
launch's average in-plan duration, measured live on the engine's stream with the device
clock: each launch's span from the end of the launch before it to its own end (dispatch
included: the interval rocprofv3 --kernel-trace reports, so the committed
profiles/*/c3_kernel_stats.csv recomputes it; k_pair's span = the scan span + the step
span; HIP events around each launch add ~2-3 us of their own and are reported as a side
figure).  The scan phase alone (`scan_phase_frac`), the inner duration (first scan
workgroup start to last end) and the whole-step fraction
`frac_step` (SURVEY 8(d) bytes per step / ms_per_step / 8 TB/s) are reported beside it.  `traffic` is the rocprofv3 PMC figure for the same workload
(profiles/pmc_traffic.json, keyed by workload, stamped with the git head it ran on).

c3 lines carry a `secondary` entry: c3nl (the same cluster without -allow-leader, whose plan
moves a different partition almost every step, unlike c3's leader 2-cycle), same steps,
warm-up and timing method, no CPU leg (--no-secondary leaves it out).

Multi-GPU: under torch.distributed.run (WORLD_SIZE set) kafkabalancer_amd.dist.bench_main;
`--gpus N` without a launcher starts N ranks itself (spawn_ranks).  Strong scaling by
default: the workload's one cluster (c3: 1M x 1000) sharded N ways, so every N runs the same
plan; --scaling weak gives every rank a full cluster.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _oracle_pl(cl):
    from oracle import oracle as O
    P = cl.n
    return O.OraclePL.from_soa(b"t", np.zeros(P + 1, np.int64), np.arange(P, dtype=np.int64),
                               cl.replica_ids, cl.replica_off, np.where(cl.weight == 0, 1.0, cl.weight),
                               np.where(cl.num_replicas == 0, np.diff(cl.replica_off), cl.num_replicas),
                               cl.set_ids, cl.set_off, cl.set_idx, cl.num_consumers)


def _move_sample(cl, cfg, seconds):
    """The oracle's move() (C restatement of steps.go:145-232, one thread like the Go
    balancer) over the first k partitions of the cluster, k grown until the sample takes
    about `seconds`: (candidates, seconds, k, leaders)."""
    from oracle import oracle as O
    O.set_threads(1)
    opl = _oracle_pl(cl)
    # ValidateWeights / ValidateReplicas / FillDefaults first (steps.go:7-66): nil Brokers
    # lists (c5's auto lists) become the default list, as before the reference's move()
    r = O.step(opl, cfg, 0x7, O.SEM_APPLIED)
    assert r["status"] == 0, r["err"]
    P = cl.n
    leaders = bool(cfg.get("allow_leader"))
    k = 1                          # (w16k: one partition's move() is ~1 s of 16384-term folds)
    while True:
        t0 = time.perf_counter()
        n, _ = O.move_sample(opl, cfg, leaders, k)
        dt = time.perf_counter() - t0
        if dt > seconds / 8 or k >= P:
            break
        k = min(P, int(k * max(2.0, (seconds / 8) / max(dt, 1e-4))))
    k2 = min(P, int(k * seconds / max(dt, 1e-6)))
    if k2 > k:
        t0 = time.perf_counter()
        n, _ = O.move_sample(opl, cfg, leaders, k2)
        dt = time.perf_counter() - t0
        k = k2
    return n, dt, k, leaders


def _plan_sample(cl, cfg, seconds, steps_max):
    """Whole Balance() steps of the plan on the oracle (balancer.go:49-65 per step, one
    thread), from the cluster's initial state, until the plan ends, steps_max steps ran
    or about `seconds` passed: (the oracle's changes, seconds)."""
    from oracle import oracle as O
    O.set_threads(1)
    opl = _oracle_pl(cl)
    out = []
    t0 = time.perf_counter()
    while len(out) < steps_max and time.perf_counter() - t0 < seconds:
        r = O.balance(opl, cfg, O.SEM_APPLIED)
        if r["status"] != 1:
            break
        out.append(r)
    return out, time.perf_counter() - t0


def cpu_baseline(cl, cfg, desc, plan_cand_per_step, seconds=12.0):
    """The reference's algorithm on the host cores: the C oracle, single
    thread like the Go balancer (kind "port"; the Go reference is not buildable here),
    on a bounded sample of the same workload:
      * c2 / c4: whole steps of the plan from the initial state (c2 ends within the budget:
        the full 100-move plan); the sample's steps are checked against the GPU engine's
        plan of the same steps, whose candidate counts are the metric's numerator;
      * c3 / c5: move() over the first k partitions (one step costs far too long on one
        core), extrapolated per candidate to ms per step with the timed plan's candidates.
    Plus the engine's own algorithm on the host (tools/cpu_engine, OpenMP) over whole steps."""
    wl = desc.get("workload")
    out = {"cores": 1, "kind": "port", "cpu_model": cpu_model(), "nproc": os.cpu_count()}
    if wl in ("c2", "c4"):
        from kafkabalancer_amd import engine as E
        och, dt = _plan_sample(cl, cfg, seconds, int(desc.get("max_reassign", 1000)))
        k = len(och)
        eng = E.Engine(cl, cfg, device=0)
        ech, err = eng.plan(k)
        cand = eng.stats()["candidates"]
        eng.close()
        same = [(c["step"], c["pidx"], c["from_"], c["to"]) for c in ech] == \
               [(c["step"], c["pidx"], c["from_"], c["to"]) for c in och]
        out.update(ms_per_step=1e3 * dt / max(k, 1), steps=k, plan_matches_gpu=same,
                   sample="oracle Balance() x %d steps of the %s plan from its initial state (%.1f s)"
                          % (k, wl, dt))
        if cand > 0:
            out.update(value=cand / dt, unit="candidates/s")
        else:
            # (c4: Remove / Add / Disallowed stages only, move() never runs: no candidates)
            out.update(value=1e3 * dt / max(k, 1), unit="ms/step")
    else:
        n, dt, k, leaders = _move_sample(cl, cfg, seconds)
        cps = n / dt
        out.update(value=cps, unit="candidates/s",
                   ms_per_step_extrapolated=1e3 * plan_cand_per_step / cps if plan_cand_per_step else None,
                   sample="oracle move(%s) over the first %d of %d partitions: %d candidates in %.1f s; "
                          "ms_per_step_extrapolated = the timed plan's candidates per step / this rate"
                          % ("leaders" if leaders else "non-leaders", k, cl.n, n, dt))
    # the engine's algorithm on the CPU (O(1) deltas + exact verification, OpenMP)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools", "cpu_engine"))
        import cpu_engine
        # every core this process may run on (OpenMP on all host cores);
        # OMP_NUM_THREADS, when set (16 on the GPU pool's boxes), is the box's share
        avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or avail
        ce = cpu_engine.CpuEngine(cl, cfg, threads=threads)
        c0 = ce.candidates()
        t0 = time.perf_counter()
        steps = 0
        while steps < 200 and time.perf_counter() - t0 < seconds:
            if ce.step() is None:
                break
            steps += 1
        dt = time.perf_counter() - t0
        val = (ce.candidates() - c0) / dt
        out["optimised_cpu"] = {"value": val, "unit": "candidates/s",
                                "ms_per_step": 1e3 * dt / max(steps, 1), "cores": threads, "steps": steps,
                                "cores_available": avail,
                                # (the GPU pool's boxes give a job OMP_NUM_THREADS = 16 of the host's
                                # cores and ask that pools stay within it: the all-cores figure is the
                                # linear extrapolation, an upper bound, not a measurement)
                                "all_cores_value_extrapolated": val * max(avail, threads) / threads,
                                "all_cores_ms_per_step_extrapolated": 1e3 * dt / max(steps, 1) * threads / max(avail, threads),
                                "all_cores_def": "value x cores_available / cores (linear scaling: an upper bound)",
                                "cores_source": "OMP_NUM_THREADS" if os.environ.get("OMP_NUM_THREADS") else "affinity",
                                "kind": "engine algorithm on the host (tools/cpu_engine, OpenMP)"}
        ce.close()
    except (ImportError, OSError, ValueError) as ex:
        out["optimised_cpu"] = {"skipped": str(ex)}
    return out


def pmc_traffic(workload, kernel):
    """HBM-side bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_bench.sh,
    tools/pmc_summarise.py): (bytes, the git head the passes ran on) or (None, None)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            d = json.load(f)
        return d[workload][kernel]["traffic_bytes_per_launch"], d[workload].get("git_head")
    except (OSError, KeyError, ValueError, TypeError):
        return None, None


def bytes_8d(cl, changes, nsets, B, rmax, full_steps):
    """SURVEY.md 8(d) algorithmic bytes of the timed steps: a full-scan step reads
    P*(8 w + 4*Rmax rep + 1 nrep + 1 want + 4 aset) + 12 B + nsets*ceil(B/64)*8; an
    early-exit stage (Remove / Add / Disallowed, steps.go:81,105,135) reads the fields
    of every fully scanned earlier stage over all P plus its own up to the hit."""
    P = cl.n
    tables = 12 * B + nsets * ((B + 63) // 64) * 8
    per = 8 + 4 * rmax + 1 + 1 + 4
    total = 0
    for c in changes:
        h = c["pidx"] + 1
        if c["step"] == "RemoveExtraReplicas":
            total += 2 * h + tables
        elif c["step"] == "AddMissingReplicas":
            total += 2 * P + 2 * h + tables
        elif c["step"] == "MoveDisallowedReplicas":
            total += 4 * P + (4 * rmax + 1 + 4) * h + tables
        else:
            total += P * per + tables
    total += (full_steps - len(changes)) * (P * per + tables)
    return total


def drop_in(args):
    """What a drop-in user pays at the workload: one line, not the headline.
    (a) kb_engine_balance per call -- the cgo shim's path, one Balance() =
    one enqueue + one synchronisation -- against the device-resident plan's per-step time;
    (b) the C++ CLI end to end on the workload's reassignment JSON (kafkabalancer.go:181-235):
    read, decode (codecs.go:15-27), kb_engine_create, the -max-reassign plan, encode
    (codecs.go:84-93), from its KB_CLI_TIMINGS phase stamps and the process wall time."""
    import subprocess
    import tempfile
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    torch.cuda.set_device(0)
    cl, cfg, desc = synth.config(args.workload, scale=args.scale)
    eng = E.Engine(cl, cfg, device=0)
    for _ in range(5):
        assert eng.balance() is not None
    n = args.steps
    t0 = time.perf_counter()
    for _ in range(n):
        if eng.balance() is None:
            break
    per_call = (time.perf_counter() - t0) / n
    # the reference's steps table walked on the host, one kb_engine_step per entry
    # (INTEGRATION.md's per-step cgo binding; ValidateWeights / ValidateReplicas /
    # FillDefaults stay Go code there and are not called here)
    walk_calls = 0
    t0 = time.perf_counter()
    for _ in range(n):
        for k in range(3, 9):
            walk_calls += 1
            if eng.step(1 << k) is not None:
                break
    per_walk = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    buf, k, rc = eng.plan_raw(n)
    plan_step = (time.perf_counter() - t0) / max(k, 1)
    eng.close()
    out = {"metric": "drop-in cost (%s)" % args.workload, "unit": "us",
           "balance_per_call_us": 1e6 * per_call, "steps_table_per_balance_us": 1e6 * per_walk,
           "steps_table_calls_per_balance": walk_calls / n,
           "plan_per_step_us": 1e6 * plan_step, "calls": n,
           "balance_def": "kb_engine_balance via ctypes, one Balance() per call (enqueue + sync), after 5 warm calls",
           "steps_table_def": "one Balance() as the reference's steps table walked on the host: kb_engine_step "
                              "per GPU step (RemoveExtraReplicas .. MoveNonLeaders) until one changes something"}
    # the CLI on the same cluster as reassignment JSON
    cli_bin = os.path.join(ROOT, "kafkabalancer_amd", "lib", "kafkabalancer")
    tmp = tempfile.mkdtemp(prefix="kbdrop")
    jpath, tpath = os.path.join(tmp, "in.json"), os.path.join(tmp, "t.json")
    try:
        t0 = time.perf_counter()
        cl.topics = None
        with open(jpath, "wb") as f:
            f.write(json.dumps(synth.to_plist(cl), separators=(",", ":")).encode())
        gen_s = time.perf_counter() - t0
        # -complete-partition defaults to true (balancer.go:30): past -max-reassign the
        # reference keeps stepping until the last partition is complete, which on c3's
        # MoveLeaders ping-pong never happens -- the drop-in run turns it off
        cmd = [cli_bin, "-input-json", "-input", jpath, "-max-reassign", str(args.cli_reassign),
               "-complete-partition=false"]
        if cfg.get("allow_leader"):
            cmd.append("-allow-leader")
        cmd += ["-min-unbalance", repr(float(cfg.get("min_unbalance", 0.01)))]
        env = dict(os.environ, KB_CLI_TIMINGS=tpath)
        t0 = time.perf_counter()
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
        wall = time.perf_counter() - t0
        assert r.returncode == 0, r.stderr[-2000:]
        with open(tpath) as f:
            ph = json.loads(f.readline())
        out["cli"] = dict(ph, wall_s=wall, cmd=" ".join(os.path.basename(c) if c == cli_bin else c for c in cmd[:1]) +
                          " " + " ".join(cmd[1:2] + ["-input", "<%.0f MB JSON>" % (ph["input_bytes"] / 1e6)] + cmd[4:]),
                          json_generation_s=gen_s,
                          plan_ms_per_change=1e3 * ph["plan_s"] / max(ph["changes"], 1))
        # the reference's default -complete-partition=true (balancer.go:30): past -max-reassign
        # the loop goes on while the change stays on the last partition, and the first change
        # elsewhere (the probe) ends it -- kb_engine_plan_until batches; with -allow-leader
        # the leader 2-cycle of SURVEY 3.4 never ends it (the reference loops forever, the
        # CLI exits 5 after max-reassign + 1e6 steps), so that case is not timed
        if cfg.get("allow_leader"):
            out["cli_default_flags"] = {"skipped": "-allow-leader: the leader 2-cycle never completes the "
                                                   "partition (the reference loops forever)"}
        else:
            cmd_d = [c for c in cmd if c != "-complete-partition=false"]
            t0 = time.perf_counter()
            r = subprocess.run(cmd_d, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
            wall_d = time.perf_counter() - t0
            assert r.returncode == 0, r.stderr[-2000:]
            with open(tpath) as f:
                ph_d = json.loads(f.read().splitlines()[-1])
            out["cli_default_flags"] = dict(ph_d, wall_s=wall_d,
                                            plan_ms_per_change=1e3 * ph_d["plan_s"] / max(ph_d["changes"], 1),
                                            vs_plan_per_step=(ph_d["plan_s"] / max(ph_d["changes"], 1)) /
                                            max(plan_step, 1e-12))
    finally:
        for q in (jpath, tpath):
            if os.path.exists(q):
                os.unlink(q)
        os.rmdir(tmp)
    out["cpu_model"] = cpu_model()
    out["nproc"] = os.cpu_count()
    print(json.dumps(out))


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: run N ranks under torch.distributed.run as a
    child process (one process per GPU, rendezvous on 127.0.0.1) and exit with its status.
    Nothing here touches the GPU: the ranks initialise their own devices."""
    import random
    import socket
    import subprocess
    # (a port below the ephemeral range: one the kernel hands out for bind(0) can be taken
    # by an outgoing connection before the launcher binds it -- EADDRINUSE, seen once)
    port = None
    for _ in range(64):
        cand = random.randrange(20000, 30000)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
            try:
                so.bind(("127.0.0.1", cand))
            except OSError:
                continue
        port = cand
        break
    if port is None:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def kernel_times(eng, steps, mode):
    """Per-kernel (us per launch, launches) over `steps` more steps of the plan, timing
    mode 1 (device clock for k_scan / k_step) or 2 (HIP events around every launch)."""
    eng.set_timing(mode)
    _, err = eng.plan(steps)
    assert err is None, err
    tk = eng.timings()
    eng.set_timing(False)
    return {k: (1e3 * v[0] / max(v[1], 1), v[1]) for k, v in tk.items()}


_T0 = time.perf_counter()


def progress(msg):
    """A line on stderr per phase (long runs -- c5, w16k, the CPU baselines -- print nothing
    else before their JSON line)."""
    print("bench %.1fs: %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--scaling", default=None, choices=[None, "weak", "strong"],
                    help="multi-GPU: strong (the default: one cluster sharded N ways) or weak (every "
                         "rank adds a full cluster)")
    ap.add_argument("--mode", default="full", choices=["full", "incremental"],
                    help="incremental: SURVEY 8(f3) rescoring mode (scans read only the blocks a "
                         "lower-bound certificate keeps); a separate line, not the full-scan roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="c3: leave out the secondary c3nl line (c3's cluster without -allow-leader)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--isolated-scan", action="store_true",
                    help="also time 200 back-to-back k_scan launches on the final state (kept out of "
                         "the default run so a rocprofv3 trace of it averages in-plan launches only)")
    ap.add_argument("--plan-out", default=None,
                    help="write the timed plan's changes (rank 0) to this JSON file")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: load the -DKB_STAMPS build and print per-phase times (not a bench line)")
    ap.add_argument("--drop-in", action="store_true",
                    help="what a drop-in user pays: kb_engine_balance per call and the CLI end to end "
                         "(decode / create / plan / encode) on the workload's JSON; a separate line")
    ap.add_argument("--cli-reassign", type=int, default=1000)
    ap.add_argument("--dist-world1", action="store_true",
                    help="test: the multi-GPU bench path (dist.bench_main, RCCL unless KB_DIST_BACKEND) "
                         "under a one-rank torch.distributed.run launch")
    ap.add_argument("--sharded", action="store_true",
                    help="one GPU: the sharded protocol (RCCL all-gather per step, plan driven from C) at "
                         "world size 1 against the plain plan over the same steps; a separate line")
    ap.add_argument("--step-alone", action="store_true",
                    help="diagnostic: k_step alone on a fixed input after the warm-up plan "
                         "(kb_engine_bench_step; with a -DKB_STOP_AT=k library: the cost up to phase k)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    if args.drop_in:
        return drop_in(args)
    if args.step_alone:
        import torch
        from kafkabalancer_amd import engine as E
        from kafkabalancer_amd import synth
        torch.cuda.set_device(0)
        cl, cfg, desc = synth.config(args.workload, scale=args.scale)
        eng = E.Engine(cl, cfg, device=0)
        _, err = eng.plan(max(args.warmup, 1))
        assert err is None, err
        steplib = os.environ.get("KB_STEP_LIB")
        if steplib:
            # a -DKB_STOP_AT=k build's k_step on this engine (same sources: same host layout);
            # the warm-up plan above ran the production library
            import ctypes
            L2 = ctypes.CDLL(steplib)
            L2.kb_engine_bench_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
            v = ctypes.c_double()
            rc = L2.kb_engine_bench_step(eng.h, args.steps, ctypes.byref(v))
            assert rc == 0, rc
            res = v.value
        else:
            res = eng.bench_step(args.steps)
        print(json.dumps({"workload": args.workload, "lib": os.path.basename(steplib or E.LIB_PATH),
                          "k_step_alone_us": res, "iters": args.steps}))
        return
    if args.stamps:
        os.environ["KB_ENGINE_LIB"] = os.environ.get("KB_STAMPS_LIB") or \
            os.path.join(ROOT, "kafkabalancer_amd", "lib", "libkbengine_stamps.so")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.dist_world1:
        from kafkabalancer_amd import dist
        return dist.bench_main(args, world, rank, local, cpu_baseline=cpu_baseline)
    if args.sharded:
        from kafkabalancer_amd import dist
        return dist.bench_world1(args)

    import torch
    torch.cuda.set_device(0)
    out = measure(args, args.workload, with_cpu=not args.no_cpu_baseline)
    if out is None:
        return
    # the plan that is not a 2-cycle: c3's cluster without -allow-leader, whose
    # 1000-step plan moves a different partition almost every step, measured the same way
    # (same steps and warm-up, no CPU leg) beside the headline
    if args.workload == "c3" and args.mode == "full" and not args.no_secondary and not args.stamps:
        sec = measure(args, "c3nl", with_cpu=False)
        r = sec["roofline"]
        out["secondary"] = {
            "workload": "c3nl", "config": sec["config"], "steps": sec["steps"], "warmup": sec["warmup"],
            "ms_per_step": sec["ms_per_step"], "device_ms_per_step": sec["config"]["device_ms_per_step"],
            "value": sec["value"], "unit": sec["unit"],
            "roofline": {k: r[k] for k in ("achieved", "peak", "unit", "frac", "avg_launch_us", "bytes_per_launch",
                                           "frac_engine_bytes", "scan_phase_us", "frac_step", "traffic")},
            "kernels_us_per_launch": sec["kernels_us_per_launch"], "engine_events": sec["engine_events"]}
    print(json.dumps(out))


def measure(args, workload, with_cpu):
    """One single-GPU bench line of `workload` (the timed plan, then the kernel-timing
    replays): the line's dict, or None for the diagnostic --stamps run (printed here)."""
    import torch
    from kafkabalancer_amd import engine as E
    from kafkabalancer_amd import synth
    cl, cfg, desc = synth.config(workload, scale=args.scale)
    progress("%s: %d partitions built" % (workload, cl.n))
    incr = args.mode == "incremental"
    eng = E.Engine(cl, cfg, device=0, time_kernels=False, incremental=incr)
    if args.warmup:
        _, err = eng.plan(args.warmup)
        assert err is None, err
    progress("engine created, %d warm-up steps" % args.warmup)
    st0 = eng.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    raw = eng.plan_raw(args.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    changes, err = eng.changes(*raw)            # (Python dicts, outside the timed region)
    assert err is None, err
    progress("timed plan: %d steps in %.3f s" % (len(changes), wall))
    st1 = eng.stats()
    if args.plan_out:
        with open(args.plan_out, "w") as f:
            json.dump(changes, f)
    steps = len(changes) + (0 if len(changes) == args.steps else 1)
    cand = st1["candidates"] - st0["candidates"]
    dev_s = st1["device_ms"] / 1e3
    ms_per_step = 1e3 * wall / max(steps, 1)
    if args.stamps:
        st = eng.stamps()
        n = max(1, eng.stats()["steps"])       # every step since the engine was created
        # (stamp ids as placed in kernels.hip; 6..20 name the fused incremental prep's phases)
        # (the fast prep, round 6, reuses the ids of the full prep's phases it replaces: 9 FP1 counts,
        # 16 FP1 marks, 19 FP1 frozen totals, 20 FP1 upper bound, 6 FP1 barrier, 0 FP2 merge,
        # 8 FP2 barrier, 10 the commit)
        names = ["prep.S+r+ubloop|fp2.merge", "step.loads", "res.reduce", "res.pred", "res.move", "res.apply(tail)",
                 "prep.P1|fp1.barrier", "pre.staged",
                 "prep.P2|fp2.barrier", "prep.P3|fp1.counts", "prep.end|fp.commit", "res.move->apply", "loads.bro+ctl",
                 "loads.rec_reduce", "loads.keys", "pre.dprep", "prep.P4|fp1.marks",
                 "eps.sync1", "eps.wave0red", "prep.positions|fp1.totals", "prep.sets|fp1.ub", "apply.loads", "apply.update"]
        counts = {"waves_scored": 7, "waves_gated_in": 15, "emits": 31, "spills": 30, "walks": 29, "walk_steps": 28, "walk_global": 27}
        mhz = 100.0 * st[25] / max(st[24], 1)           # shader clock (the phase stamps' unit)
        names = names + ["loads.broker", None, None, "stamp.overhead", "loads.setbits", "loads.hdr"]
        print(json.dumps({"k_step_clock_mhz": mhz,
                          "k_step_us": st[24] / 100.0 / n,
                          "stamps_us_per_step": {k: st[i] / mhz / n for i, k in enumerate(names) if k},
                          "counts_per_step": {k: st[i] / n for k, i in counts.items()},
                          "stats": eng.stats()}))
        return None
    eng.close()
    # per-kernel durations, outside the headline timing, over the SAME steps of the plan as
    # the headline: a fresh engine replays the warm-up and the timed steps (the plan is
    # deterministic), so the kernel figures describe the timed steps and a rocprofv3 trace
    # of this command averages over those steps only (every stretch covers steps 0..W+K).
    # (a) the device clock (scan workgroups and k_step stamp the 100 MHz clock): each
    # launch's span from the end of the kernel before it to its own end -- dispatch
    # included, the interval rocprofv3 --kernel-trace reports, so the scan + step spans add
    # up to the step time (the roofline's figure) -- and the inner interval, first workgroup
    # start .. last end; (b) HIP events around every launch (each event adds its own
    # ~2-3 us: an upper bound, a side figure), on a third replay
    kt_steps = steps

    def replay(mode):
        e = E.Engine(cl, cfg, device=0, time_kernels=False, incremental=incr)
        if args.warmup:
            _, err2 = e.plan(args.warmup)
            assert err2 is None, err2
        s0 = e.stats()
        kt = kernel_times(e, kt_steps, mode)
        s1 = e.stats()
        iso = e.bench_scan(200) if (mode == 1 and args.isolated_scan) else None
        e.close()
        return kt, s0, s1, iso

    kdc, stk0, stk1, scan_iso_us = replay(1)
    progress("kernel timing replay (device clock) done")
    kev, _, _, _ = replay(2)
    progress("kernel timing replay (events) done")
    scan_us, scan_n = kdc["scan"]
    if not scan_n:                      # (no back-to-back launch: the inner interval)
        scan_us, scan_n = kdc["scan_inner"]
    scan_clock_us = kdc["scan_inner"][0]
    bytes_scan = st1["scan_bytes"]
    if incr:
        # bytes the incremental scans actually read: their blocks' partition words
        # (+ the 16-B block descriptors), per scan launch of the events stretch
        per_part = bytes_scan / max(cl.n, 1)
        nscans = max(kdc["scan_inner"][1], 1)
        blk = stk1["blocks_scanned"] - stk0["blocks_scanned"]
        bytes_scan = blk * 128 * per_part / nscans + 16 * blk / nscans
    achieved = bytes_scan / (scan_us * 1e-6) / 1e9
    rmax = st1["max_replicas"]
    b8d = bytes_8d(cl, changes, st1["n_sets"], st1["n_brokers"], rmax, steps)
    whole_gbs = b8d / max(wall, 1e-12) / 1e9
    early_exit = any(c["step"] in ("RemoveExtraReplicas", "AddMissingReplicas", "MoveDisallowedReplicas")
                     for c in changes)
    weights = "Zipf-like weights w = r^-1.1, r ~ U[1, 1e6]" if desc.get("weights") == "zipf" else \
        "weights absent (FillDefaults -> 1.0: uniform, exact ties)"
    # fused pairs (k_pair: the scan's grid plus the step workgroup in one launch): the launch
    # rocprofv3 sees is the whole step, so the roofline is priced on it -- its duration is the
    # scan span plus the step span -- and the scan phase inside it is a side figure
    fused = bool(st1.get("fused_pairs")) and not incr
    kname = "k_pair" if fused else "k_scan"
    scan_phase_us = scan_us
    pair_timing = None
    if fused:
        if kdc.get("step", (0, 0))[1] and kdc.get("scan", (0, 0))[1]:
            scan_us = kdc["scan"][0] + kdc["step"][0]
            pair_timing = "spans"
        elif kdc.get("pair", (0, 0))[1]:
            # (no back-to-back spans -- c5's bound passes sit between the launches: the launch
            # from its first workgroup's start to the step workgroup's end, dispatch excluded)
            scan_us = kdc["pair"][0]
            pair_timing = "first workgroup start .. step end"
        achieved = bytes_scan / (scan_us * 1e-6) / 1e9
    traffic, traffic_git = (None, None) if incr else pmc_traffic(workload, kname)
    # achieved = SURVEY.md 8(d)'s algorithmic bytes of a step (P * (8 w + 4 Rmax rep + 1 nrep +
    # 1 want + 4 aset) + 12 B + the allowed-set words; early-exit stages to their hit) / the
    # launch's duration; the engine's own layout (18 B per partition at RF 3) beside it.
    # (incremental mode: the blocks its scans read, engine layout -- never the full-scan figure)
    bytes_alg = bytes_scan if incr else b8d / max(steps, 1)
    achieved = bytes_alg / (scan_us * 1e-6) / 1e9
    achieved_eng = bytes_scan / (scan_us * 1e-6) / 1e9
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": kname + (" (one launch per step: the scan's grid and the step workgroup)" if fused else ""),
            "bytes_per_launch": bytes_alg,
            "bytes_per_launch_def": ("SURVEY.md 8(d) algorithmic bytes per step (one launch per step): "
                                     "P*(8 w + 4*%d rep + 1 nrep + 1 want + 4 aset) + 12 B + nsets*ceil(B/64)*8"
                                     % rmax) if not incr else
                                    ("engine layout: per partition 8 w + 4 meta + 2*%d rep x the blocks the "
                                     "incremental scans read (+16 B per block descriptor); the full scan reads %d"
                                     % (rmax, st1["scan_bytes"])),
            "achieved_engine_bytes": achieved_eng, "frac_engine_bytes": achieved_eng / HBM_PEAK_GBS,
            "engine_bytes_per_launch": bytes_scan,
            "engine_bytes_def": "the engine's layout: per partition 8 w + 4 meta + 2*%d rep" % rmax,
            "avg_launch_us": scan_us,
            "timing": (("device clock (100 MHz), in-plan launches back to back: the previous launch's end "
                        "to the step workgroup's end (dispatch included, the interval rocprofv3 "
                        "--kernel-trace reports), %d launches" % scan_n) if pair_timing == "spans" else
                       ("device clock (100 MHz): k_pair's first workgroup start to its step workgroup's "
                        "end (dispatch excluded: no back-to-back launches), %d launches" % kdc["pair"][1])) if fused else
                      ("device clock (100 MHz), in-plan launches back to back: the previous k_step's end "
                       "to the last scan workgroup's end (dispatch included, the interval rocprofv3 "
                       "--kernel-trace reports), %d launches" % scan_n),
            "avg_launch_us_device_clock": scan_clock_us,
            "device_clock_def": "first scan workgroup start .. last end (no dispatch)",
            "frac_device_clock": bytes_alg / (scan_clock_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "scan_phase_us": scan_phase_us,
            "scan_phase_frac": bytes_alg / (scan_phase_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "scan_phase_def": "the scan's span alone: the previous step's end to the last scan workgroup's "
                              "end (device clock)",
            "avg_launch_us_events": kev["scan"][0],
            "events_def": "HIP events around every launch (each event adds its own time: an upper bound)",
            "frac_step": whole_gbs / HBM_PEAK_GBS,
            "frac_step_def": "SURVEY.md 8(d) algorithmic bytes of the timed steps / their wall time / 8 TB/s"
                             + (" (early-exit stages counted to their hit: ms_per_step is the headline, "
                                "GB/s informational)" if early_exit else ""),
            "bytes_8d_per_step": b8d / max(steps, 1),
            "traffic_source": "profiles/pmc_traffic.json[%s] (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per "
                              "launch, separate passes)" % workload,
            "traffic_git_head": traffic_git}
    if scan_iso_us is not None:
        roof.update(avg_launch_us_isolated=scan_iso_us,
                    frac_isolated=bytes_alg / (scan_iso_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                    isolated_timing="HIP events around 200 back-to-back k_scan launches on the final state")
    out = {
        "metric": "candidate moves scored/sec (+ ms per reassignment step)",
        "value": cand / wall,
        "unit": "candidates/s",
        "n_gpus": 1,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (numpy PCG64 seed %#x), %s" % (synth.SEEDS[workload], weights),
        "config": dict(desc, parallelism="single-gpu", device_ms_per_step=1e3 * dev_s / max(steps, 1),
                       mode=args.mode, fused_pairs=fused),
        "roofline": roof,
        "kernels_us_per_launch": {k: v[0] for k, v in kdc.items() if v[1]},
        "kernels_launches": {k: v[1] for k, v in kdc.items() if v[1]},
        "kernels_us_per_launch_events": {k: v[0] for k, v in kev.items() if v[1]},
        "incremental": ({"blocks_per_scan": (stk1["blocks_scanned"] - stk0["blocks_scanned"]) / max(kdc["scan_inner"][1], 1),
                         "blocks_total": (cl.n + 127) // 128} if incr else None),
        "kernel_timing_steps": kt_steps,
        "kernel_timing_def": "fresh engines replay the warm-up and the same %d timed steps (device clock, then "
                             "HIP events); every kernel figure describes the timed steps" % kt_steps,
        "engine_events": {k: st1[k] - st0[k] for k in ("retries", "refreshes", "exact_halts", "exact_folds")},
    }
    if with_cpu:
        progress("CPU baseline (%.0f s sample)" % args.cpu_seconds)
        out["cpu_baseline"] = cpu_baseline(cl, cfg, desc, cand / max(steps, 1), args.cpu_seconds)
        progress("CPU baseline done")
        cb = out["cpu_baseline"]
        if cb.get("unit") == "candidates/s" and cb.get("value"):
            out["speedup_vs_cpu"] = out["value"] / cb["value"]
        elif cb.get("unit") == "ms/step":
            out["speedup_vs_cpu"] = cb["value"] / ms_per_step
    return out


if __name__ == "__main__":
    sys.exit(main() or 0)
