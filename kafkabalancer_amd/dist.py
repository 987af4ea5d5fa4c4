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
    def __init__(self, engine, world, device_tensors=True, group=None):
        import torch
        self.engine = engine
        self.world = world
        self.group = group
        nb = engine.summary_bytes()
        dev = "cuda" if device_tensors else "cpu"
        self.summary = torch.zeros(nb, dtype=torch.uint8, device=dev)
        self.gathered = torch.zeros(world * nb, dtype=torch.uint8, device=dev)
        self.parts = list(self.gathered.chunk(world))

    def step(self):
        import torch.distributed as dist
        while True:
            self.engine.step_begin(self.summary)
            if self.summary.is_cuda:
                dist.all_gather_into_tensor(self.gathered, self.summary, group=self.group)
            else:
                dist.all_gather(self.parts, self.summary, group=self.group)
            ch = self.engine.step_finish(self.gathered, self.world)
            # "retry": the bounds could not decide on approximate loads; every rank
            # refolded its loads exactly and the step runs again
            if not (isinstance(ch, str) and ch == "retry"):
                return ch

    def plan(self, steps):
        out = []
        for _ in range(steps):
            ch = self.step()
            if ch is None:
                break
            out.append(ch)
        return out


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


def bench_main(args, world, rank, local):
    """bench.py for N > 1 (launched by torch.distributed.run)."""
    import torch
    import torch.distributed as dist
    from . import engine as E
    from . import synth
    torch.cuda.set_device(local)
    dist.init_process_group("nccl")
    # weak scaling: 1M partitions per GPU (c3 shape), the same seed on every rank
    cl, cfg, desc = synth.config(args.workload, scale=args.scale * world)
    begin, end = shard_bounds(cl.n, world, rank)
    eng = E.Engine(cl, cfg, device=local, shard=(begin, end))
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    sp = ShardedPlanner(_DeviceEngineAdapter(eng), world, device_tensors=True)
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
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    wall = float(dt.item())
    st1 = eng.stats()
    steps = max(1, len(changes))
    cand = st1["candidates"] - st0["candidates"]       # merged counts: the whole job
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (numpy PCG64), Zipf weights r^-1.1",
            "config": dict(desc, parallelism="partition-sharded x%d, replicated broker state, "
                                              "1 all-gather per step" % world),
        }
        print(json.dumps(out))
    eng.close()
    dist.destroy_process_group()
