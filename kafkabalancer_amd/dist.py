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


def bench_main(args, world, rank, local):
    """bench.py for N > 1 (launched by torch.distributed.run)."""
    import torch
    import torch.distributed as dist
    from . import engine as E
    from . import synth
    import os
    # KB_DIST_BACKEND=gloo: rehearsal with host-staged summaries (ranks may share a GPU)
    backend = os.environ.get("KB_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(backend)
    # strong scaling (c5 default, BASELINE configs[4]): one cluster of the configured size
    # sharded N ways; weak: every rank adds a full cluster's worth of partitions
    scaling = getattr(args, "scaling", None) or ("strong" if args.workload == "c5" else "weak")
    cl, cfg, desc = synth.config(args.workload, scale=args.scale * (world if scaling == "weak" else 1))
    begin, end = shard_bounds(cl.n, world, rank)
    eng = E.Engine(cl, cfg, device=local, shard=(begin, end))
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    sp = ShardedPlanner(_DeviceEngineAdapter(eng), world, device_tensors=True, staged=backend != "nccl")
    sp.plan(args.warmup)
    st0 = eng.stats()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    changes = sp.plan(args.steps)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    if rank == 0 and getattr(args, "plan_out", None):
        with open(args.plan_out, "w") as f:
            json.dump(changes, f)
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    wall = float(dt.item())
    st1 = eng.stats()
    steps = max(1, len(changes))
    cand = st1["candidates"] - st0["candidates"]       # merged counts: the whole job
    # per-kernel device-clock durations over a second stretch (this rank's shard)
    eng.set_timing(True)
    sp.plan(min(args.steps, 100))
    tk = eng.timings()
    scan_ms, scan_n = tk["scan_inner"]     # (first workgroup start .. last end; the summary and
                                          # the all-gather sit between the scan and k_step)
    scan_us = 1e3 * scan_ms / max(scan_n, 1)
    shard_bytes = st1["scan_bytes"]
    achieved = shard_bytes / (scan_us * 1e-6) / 1e9 if scan_us > 0 else 0.0
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
            "data": "synthetic (numpy PCG64), %s" % ("Zipf weights r^-1.1" if desc.get("weights") == "zipf"
                                                      else "uniform weights"),
            "config": dict(desc, parallelism="partition-sharded x%d, replicated broker state, "
                                              "1 all-gather per step" % world),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": None, "kernel": "k_scan (rank 0 shard)",
                         "bytes_per_launch": shard_bytes, "avg_launch_us": scan_us,
                         "timing": "device clock: earliest workgroup start to latest workgroup end"},
            "kernels_us_per_launch": {k: 1e3 * v[0] / max(v[1], 1) for k, v in tk.items() if v[1]},
            "exchange": backend,
        }
        print(json.dumps(out))
    eng.close()
    dist.destroy_process_group()
