"""Multi-GPU plan driver: one process per GPU, partitions sharded, one
all-gather of a fixed-size per-rank summary per step.

Every rank holds the full cluster (the exact partition-ordered load refolds
need it) and scans only partitions [shard_begin, shard_end).  A step is:

    engine.step_begin(summary)            # prep, set lists, scan, near-tie census (local)
    all_gather(gathered, summary)         # RCCL over xGMI (gloo on CPU tests)
    change = engine.step_finish(gathered) # merge + identical resolve/apply on every rank

`ShardedPlanner` is written against a tiny engine protocol (summary_bytes,
step_begin, step_finish) so the exchange logic is testable with a CPU engine
over gloo (tests/test_dist.py).
"""
import json
import os
import time

TILE = 1024


def shard_bounds(n, world, rank):
    """Contiguous shards aligned to the engine's 1024-partition tiles."""
    per = -(-n // world)
    per = -(-per // TILE) * TILE
    begin = min(n, rank * per)
    end = min(n, begin + per)
    return begin, end


class ShardedPlanner:
    """staged=True: device summaries exchanged through host copies over gloo (rehearsal
    of the N-rank protocol on a box whose ranks share one GPU; RCCL needs one GPU per rank)."""

    def __init__(self, engine, world, device_tensors=True, group=None, staged=False):
        import torch
        self.engine = engine
        self.world = world
        self.group = group
        self.staged = staged
        self.dev = "cuda" if device_tensors else "cpu"
        self._alloc()

    def _alloc(self):
        """Exchange buffers of the engine's current summary size (it grows when a rank
        summary overflows: every rank sees the same flags and grows alike)."""
        import torch
        nb = self.engine.summary_bytes()
        world = self.world
        self.summary = torch.zeros(nb, dtype=torch.uint8, device=self.dev)
        self.gathered = torch.zeros(world * nb, dtype=torch.uint8, device=self.dev)
        self.parts = list(self.gathered.chunk(world))
        if self.staged:
            self.h_summary = torch.zeros(nb, dtype=torch.uint8)
            self.h_gathered = torch.zeros(world * nb, dtype=torch.uint8)
            self.h_parts = list(self.h_gathered.chunk(world))
        if self.dev == "cuda":
            torch.cuda.synchronize()

    def step(self):
        import torch
        import torch.distributed as dist
        while True:
            self.engine.step_begin(self.summary)
            if self.staged:
                torch.cuda.synchronize()
                self.h_summary.copy_(self.summary)
                dist.all_gather(self.h_parts, self.h_summary, group=self.group)
                self.gathered.copy_(self.h_gathered)
                torch.cuda.synchronize()
            elif self.summary.is_cuda:
                dist.all_gather_into_tensor(self.gathered, self.summary, group=self.group)
            else:
                dist.all_gather(self.parts, self.summary, group=self.group)
            ch = self.engine.step_finish(self.gathered, self.world)
            # "retry": the bounds could not decide on approximate loads; every rank
            # refolded its loads exactly and the step runs again; "grow": a rank summary
            # overflowed, the summaries grew and the step runs again
            if isinstance(ch, str) and ch == "grow":
                self._alloc()
                continue
            if not (isinstance(ch, str) and ch == "retry"):
                return ch

    def plan(self, steps, batch=64):
        """`steps` merged steps; engines with the batched protocol (sharded_*) enqueue
        `batch` rounds (scan, summary, all-gather, resolve) per host round trip."""
        if not hasattr(self.engine, "sharded_collect"):
            out = []
            for _ in range(steps):
                ch = self.step()
                if ch is None:
                    break
                out.append(ch)
            return out
        import torch
        import torch.distributed as dist
        out = []
        while len(out) < steps:
            b = min(batch, steps - len(out))
            self.engine.sharded_reset(b)
            for _ in range(b):
                self.engine.sharded_scan(self.summary)
                if self.staged:
                    torch.cuda.synchronize()
                    self.h_summary.copy_(self.summary)
                    dist.all_gather(self.h_parts, self.h_summary, group=self.group)
                    self.gathered.copy_(self.h_gathered)
                    torch.cuda.synchronize()
                else:
                    dist.all_gather_into_tensor(self.gathered, self.summary, group=self.group)
                self.engine.sharded_resolve(self.gathered, self.world)
            status, changes = self.engine.sharded_collect(b + 1)
            out.extend(changes)
            if status == "done":
                break
            if status == "grow":
                self._alloc()
        return out[:steps]


class _DeviceEngineAdapter:
    """Engine (C ABI) -> tensor-based protocol used by ShardedPlanner."""

    def __init__(self, eng):
        self.eng = eng

    def summary_bytes(self):
        return self.eng.summary_bytes()

    def step_begin(self, summary):
        self.eng.step_begin(summary.data_ptr())

    def step_finish(self, gathered, world):
        return self.eng.step_finish(gathered.data_ptr(), world)

    def sharded_reset(self, budget):
        self.eng.sharded_reset(budget)

    def sharded_scan(self, summary):
        self.eng.sharded_scan(summary.data_ptr())

    def sharded_resolve(self, gathered, world):
        self.eng.sharded_resolve(gathered.data_ptr(), world)

    def sharded_collect(self, cap):
        return self.eng.sharded_collect(cap)


def _timed(fn, steps):
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn(steps)
    torch.cuda.synchronize()
    return out, time.perf_counter() - t0


def _rccl_engine(E, cl, cfg, local, shard, world, rank, uid):
    eng = E.Engine(cl, cfg, device=local, shard=shard)
    eng.comm_init(world, rank, uid)
    return eng


def _plan_or_raise(fn, steps):
    changes, err = fn(steps)
    if err is not None:
        raise err
    return changes


def bench_main(args, world, rank, local, cpu_baseline=None):
    """bench.py for N > 1 (launched by torch.distributed.run).  With RCCL (the default) the
    whole plan runs in C: kb_engine_sharded_plan enqueues 64 rounds of (scan + rank summary,
    ncclAllGather on the engine's stream, resolve) per host round trip; the communicator's
    unique id goes from rank 0 to the others over torch.distributed.  KB_DIST_BACKEND=gloo:
    the host-staged rehearsal (ShardedPlanner, ranks may share a GPU)."""
    import torch
    import torch.distributed as dist
    from . import engine as E
    from . import synth
    import os
    backend = os.environ.get("KB_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(backend)
    # strong scaling (the default): the workload's one cluster (c3: BASELINE's 1M x 1000)
    # sharded N ways, so the N-GPU line is the same plan as the 1-GPU line; weak: every rank
    # adds a full cluster's worth of partitions (--scaling weak)
    scaling = getattr(args, "scaling", None) or "strong"
    cl, cfg, desc = synth.config(args.workload, scale=args.scale * (world if scaling == "weak" else 1))
    shard = shard_bounds(cl.n, world, rank)
    rccl = backend == "nccl"

    def make():
        if rccl:
            # a fresh RCCL unique id per communicator: the bootstrap root behind an id serves
            # one ncclCommInitRank round (the kernel-timing replay below builds a second one)
            box = [E.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            e = _rccl_engine(E, cl, cfg, local, shard, world, rank, box[0])
            return e, (lambda n: _plan_or_raise(e.sharded_plan, n))
        e = E.Engine(cl, cfg, device=local, shard=shard)
        e.set_stream(torch.cuda.current_stream().cuda_stream)
        sp = ShardedPlanner(_DeviceEngineAdapter(e), world, device_tensors=True, staged=True)
        return e, sp.plan

    eng, plan = make()
    plan(args.warmup)
    st0 = eng.stats()
    torch.cuda.synchronize()
    dist.barrier()
    changes, wall_r = _timed(plan, args.steps)
    dist.barrier()
    torch.cuda.synchronize()
    if rank == 0 and getattr(args, "plan_out", None):
        with open(args.plan_out, "w") as f:
            json.dump(changes, f)
    dt = torch.tensor([wall_r], dtype=torch.float64, device="cuda" if rccl else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    wall = float(dt.item())
    st1 = eng.stats()
    steps = max(1, len(changes))
    cand = st1["candidates"] - st0["candidates"]       # merged counts: the whole job
    dev_ms = st1["device_ms"] if rccl else None        # (the timed plan call's device time)
    eng.close()
    # per-kernel device-clock durations over the same steps (a fresh engine replays the
    # warm-up and the timed steps): the scan launch's span, as on one GPU -- the end of
    # the kernel before it (the last round's k_step) to the last scan workgroup's end
    eng, plan = make()
    plan(args.warmup)
    eng.set_timing(True)
    plan(steps)
    tk = eng.timings()
    eng.close()
    dist.barrier()
    scan_ms, scan_n = tk["scan"]
    timing = "device clock: the previous round's k_step end to the last scan workgroup's end (dispatch included)"
    if not scan_n:
        scan_ms, scan_n = tk["scan_inner"]
        timing = "device clock: earliest scan workgroup start to latest end"
    scan_us = 1e3 * scan_ms / max(scan_n, 1)
    shard_bytes = st1["scan_bytes"]
    scan_achieved = shard_bytes / (scan_us * 1e-6) / 1e9 if scan_us > 0 else 0.0
    # the same pricing as the 1-GPU line: SURVEY 8(d)'s algorithmic bytes of a step over the
    # step's device time -- here one round (scan + rank summary, the all-gather, the resolve)
    # of the whole cluster on N GPUs, against N x the HBM peak (dev_ms: the timed call's
    # device time on rank 0; every rank runs the same rounds)
    b8d = cl.n * (8 + 4 * st1["max_replicas"] + 1 + 1 + 4) + 12 * st1["n_brokers"] + \
        st1["n_sets"] * ((st1["n_brokers"] + 63) // 64) * 8
    round_us = 1e3 * (dev_ms if dev_ms else wall * 1e3) / steps
    achieved = b8d / (round_us * 1e-6) / 1e9
    tr1, tr_src = _round_traffic(args.workload)
    if rank == 0:
        out = {
            "metric": "candidate moves scored/sec (+ ms per reassignment step)",
            "value": cand / wall,
            "unit": "candidates/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * wall / steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (numpy PCG64 seed %#x), %s" % (synth.SEEDS[args.workload],
                                                             "Zipf weights r^-1.1" if desc.get("weights") == "zipf"
                                                             else "uniform weights"),
            "config": dict(desc, parallelism="partition-sharded x%d, replicated broker state, "
                                              "1 all-gather per step (%s)" % (world, "RCCL, plan driven from C"
                                                                              if rccl else "gloo, host-staged")),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0 * world, "unit": "GB/s",
                         "frac": achieved / (8000.0 * world),
                         # (PMC passes are 1-GPU runs: the world-1 sharded round's k_scansum + k_step,
                         # tools/pmc_sharded.sh; at N > 1 a rank scans 1/N of it, so only the world-1
                         # line carries it as its traffic, the others beside it)
                         "traffic": tr1 if world == 1 else None,
                         "traffic_world1_round": tr1, "traffic_source": tr_src,
                         "kernel": "one sharded round: k_scansum (scan + rank summary) + ncclAllGather + k_step "
                                   "(resolve), whole cluster on %d GPUs" % world,
                         "bytes_per_launch": b8d,
                         "bytes_per_launch_def": "SURVEY.md 8(d) algorithmic bytes of one step of the whole cluster",
                         "avg_launch_us": round_us,
                         "timing": "device time of the timed plan call (rank 0) / steps" if dev_ms else
                                   "wall time / steps (no device time on this path)",
                         "scan_span_us": scan_us, "scan_timing": timing, "scan_launches": scan_n,
                         "scan_bytes_per_rank": shard_bytes,
                         "scan_achieved_per_rank": scan_achieved, "scan_frac_per_rank": scan_achieved / 8000.0,
                         "frac_step": b8d / (wall / steps) / 8e12,
                         "frac_step_def": "SURVEY.md 8(d) bytes of the whole cluster per step / ms_per_step / 8 TB/s"},
            "kernels_us_per_launch": {k: 1e3 * v[0] / max(v[1], 1) for k, v in tk.items() if v[1]},
            "kernel_timing_def": "a fresh engine per rank replays the warm-up and the same timed steps",
            "exchange": "rccl" if rccl else backend,
        }
        if cpu_baseline is not None and not getattr(args, "no_cpu_baseline", False):
            out["cpu_baseline"] = cpu_baseline(cl, cfg, desc, cand / steps, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def _round_traffic(workload):
    """HBM-side bytes of one world-1 sharded round (k_scansum + k_step) from the committed
    PMC passes (profiles/pmc_traffic.json["<workload>_sharded"]): (bytes, source) or (None, None)."""
    try:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        with open(os.path.join(root, "profiles", "pmc_traffic.json")) as f:
            d = json.load(f)[workload + "_sharded"]
        b = d["k_scansum"]["traffic_bytes_per_launch"] + d["k_step"]["traffic_bytes_per_launch"]
        return b, "profiles/pmc_traffic.json[%s_sharded] (k_scansum + k_step per round, git %s)" % (
            workload, d.get("git_head"))
    except (OSError, KeyError, ValueError, TypeError):
        return None, None


def bench_world1(args, cpu_baseline=None):
    """`bench.py --sharded` (one GPU): the sharded protocol at world size 1 -- a shard of
    every partition, kb_engine_sharded_plan with a one-rank RCCL communicator -- against the
    plain plan (kb_engine_plan) over the same steps: the protocol's own overhead per step
    (the extra launches, the all-gather, the unfused resolve).  One JSON line; not the
    headline."""
    import torch
    from . import engine as E
    from . import synth
    torch.cuda.set_device(0)
    cl, cfg, desc = synth.config(args.workload, scale=args.scale)
    uid = E.comm_unique_id()
    eng = _rccl_engine(E, cl, cfg, 0, (0, cl.n), 1, 0, uid)
    _plan_or_raise(eng.sharded_plan, args.warmup)
    (buf, n, rc), wall_s = _timed(eng.sharded_plan_raw, args.steps)
    sh_changes, err = eng.changes(buf, n, rc)
    assert err is None, err
    sh_stats = eng.stats()
    eng.close()
    ref = E.Engine(cl, cfg, device=0)
    _plan_or_raise(ref.plan, args.warmup)
    (buf, n, rc), wall_p = _timed(ref.plan_raw, args.steps)
    pl_changes, err = ref.changes(buf, n, rc)
    assert err is None, err
    fused = ref.stats()["fused_pairs"]
    ref.close()
    key = lambda ch: [(c["step"], c["pidx"], c["from_"], c["to"], c["slot"]) for c in ch]
    steps = max(1, len(sh_changes))
    out = {"metric": "sharded protocol at world size 1 (%s)" % args.workload, "unit": "ms/step",
           "ms_per_step_sharded": 1e3 * wall_s / steps, "ms_per_step_plain": 1e3 * wall_p / max(1, len(pl_changes)),
           "ratio": (wall_s / steps) / (wall_p / max(1, len(pl_changes))), "steps": steps, "warmup": args.warmup,
           "plans_equal": key(sh_changes) == key(pl_changes), "plain_fused_pairs": fused,
           "sharded_stats": {k: sh_stats.get(k) for k in ("refreshes", "exact_halts", "exact_folds", "retries",
                                                         "spill_grows", "eager", "fast_preps", "relists")},
           "def": "kb_engine_sharded_plan (scan + k_summary, ncclAllGather on a 1-rank communicator, k_step "
                  "resolve; 64 rounds per host round trip) vs kb_engine_plan, same warm-up and steps"}
    print(json.dumps(out), flush=True)
