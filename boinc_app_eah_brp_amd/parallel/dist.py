"""Template-bank sharding over torch.distributed (RCCL on MI355X, gloo on CPU).

The reference is a single-process, single-device application; Einstein@Home
parallelises by handing work units to different volunteer hosts
(erp_boinc_wrapper.cpp:487-584). On an 8x MI355X node one work unit is
split instead: each rank processes a contiguous block of the template bank on
its own GPU, and the per-rank 5x100 candidate tables (24 000 bytes each) are
exchanged with ONE all-gather over xGMI and merged in rank order.

The merge is exact: per harmonic level the sequential search
keeps the 100 distinct bins with the largest maximum power, tagged with the
first template reaching it, and `CandidateTable.merge` of tables ordered by
template range yields the same table (up to exact power ties at the 100th
place, where the reference's qsort order is itself unspecified).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .. import native

TABLE_BYTES = 24000  # 500 x 48-byte CP_cand


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: object = None  # torch.device of the collectives

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_distributed(backend: str | None = None) -> DistContext:
    """Initialise torch.distributed from the torchrun environment (no-op for one process)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return DistContext(rank=0, world=1, local_rank=local, backend="none")
    import torch
    import torch.distributed as dist

    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        kwargs = {}
        if backend == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return DistContext(rank=rank, world=world, local_rank=local, backend=backend, device=dev)


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of templates for `rank` (earlier ranks get earlier templates)."""
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def allgather_tables(table, ctx: DistContext) -> list:
    """All-gather every rank's candidate table (24 KB) with one collective."""
    brp = native()
    if not ctx.distributed:
        return [table]
    import torch
    import torch.distributed as dist

    mine = torch.from_numpy(np.asarray(table.to_bytes(), dtype=np.uint8).copy())
    mine = mine.to(ctx.device)
    out = torch.empty(ctx.world * TABLE_BYTES, dtype=torch.uint8, device=ctx.device)
    dist.all_gather_into_tensor(out, mine)
    host = out.cpu().numpy()
    tables = []
    for r in range(ctx.world):
        t = brp.CandidateTable()
        t.from_bytes(np.ascontiguousarray(host[r * TABLE_BYTES:(r + 1) * TABLE_BYTES]))
        tables.append(t)
    return tables


def merge_tables(tables) -> object:
    """Merge per-shard tables given in template-range order."""
    brp = native()
    out = brp.CandidateTable()
    for t in tables:
        out.merge(t)
    return out


def barrier(ctx: DistContext) -> None:
    if ctx.distributed:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(value: float, ctx: DistContext) -> float:
    if not ctx.distributed:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class ShardedSearch:
    """One work unit searched by all ranks: rank r takes templates shard_range(r)."""

    def __init__(self, options: dict, ctx: DistContext, device: int | None = None, use_cpu: bool = False,
                 streams: int = 1):
        """`streams` independent pipelines (HIP stream + buffers) share this rank's
        GPU: while the host applies one batch's candidates the GPU runs the next."""
        self.brp = native()
        self.ctx = ctx
        self.options = dict(options)
        if use_cpu:
            self.options["use_cpu"] = True
        dev = ctx.local_rank if device is None else device
        streams = max(1, streams)
        self.session = self.brp.SearchSession()
        self.session.open(self.options, streams, [] if use_cpu else [dev] * streams)
        self.total = self.session.total()
        self.begin, self.end = shard_range(self.total, ctx.rank, ctx.world)
        self.timings: dict = {}  # accumulated seconds per phase of step()

    def step(self, limit: int | None = None):
        """Whiten + search this rank's shard + all-gather + merge. Returns the merged table."""
        import time

        total = self.total if limit is None else min(limit, self.total)
        begin, end = shard_range(total, self.ctx.rank, self.ctx.world)
        t0 = time.perf_counter()
        self.session.prepare()
        t1 = time.perf_counter()
        table, _ = self.session.run(begin, end, self.brp.CandidateTable())
        t2 = time.perf_counter()
        tables = allgather_tables(table, self.ctx)
        merged = merge_tables(tables)
        t3 = time.perf_counter()
        for k, v in (("prepare", t1 - t0), ("templates", t2 - t1), ("merge", t3 - t2)):
            self.timings[k] = self.timings.get(k, 0.0) + v
        return merged

    def write_output(self, table, n_done: int | None = None):
        """Rank 0 writes the checkpoint/result files of the merged table."""
        if self.ctx.rank != 0:
            return
        self.brp.finalize_output(self.options, self.session.geometry(),
                                 self.total if n_done is None else n_done, table)
