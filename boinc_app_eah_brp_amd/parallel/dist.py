"""Template-bank sharding over torch.distributed (RCCL on MI355X, gloo on CPU).

The reference is a single-process, single-device application; Einstein@Home
parallelises by handing work units to different volunteer hosts
(erp_boinc_wrapper.cpp:487-584). On an 8x MI355X node one work unit is
split instead: each rank processes a contiguous block of the template bank on
its own GPU, and the per-rank 5x100 candidate tables (24 000 bytes each) are
exchanged with ONE all-gather over xGMI and merged in rank order.

Failure handling: every collective runs under
BRP_COLLECTIVE_TIMEOUT seconds (default 600). When one fails or times out the
rank aborts its process group, logs the failure and degrades to a single-GPU
search: it computes the other ranks' shards itself, so rank 0 still writes the
full, exact result. `BRP_FAULT=collective_timeout[:R]` makes rank R (default 1)
stall before its first all-gather to exercise that path.

The merge is exact: per harmonic level the sequential search
keeps the 100 distinct bins with the largest maximum power, tagged with the
first template reaching it, and `CandidateTable.merge` of tables ordered by
template range yields the same table (up to exact power ties at the 100th
place, where the reference's qsort order is itself unspecified).
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from datetime import timedelta

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
    degraded: bool = False  # a collective failed: this rank now searches alone
    stalled: bool = False   # the collective_timeout fault already fired
    solo_shard: bool = False  # one process times rank `rank`'s shard of a `world`-rank run (no collectives)

    @property
    def distributed(self) -> bool:
        return self.world > 1 and not self.degraded and not self.solo_shard


class CollectiveError(RuntimeError):
    """A collective failed or exceeded BRP_COLLECTIVE_TIMEOUT."""


def collective_timeout_s() -> float:
    return float(os.environ.get("BRP_COLLECTIVE_TIMEOUT", "600"))


def fault_param(name: str) -> str | None:
    """Parameter of `name` in BRP_FAULT ("" if given without one), None if absent
    (same syntax as csrc/core/fault.hpp)."""
    for tok in os.environ.get("BRP_FAULT", "").split(","):
        key, _, arg = tok.partition(":")
        if key == name:
            return arg
    return None


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
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=timedelta(seconds=collective_timeout_s()), **kwargs)
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
    stall = fault_param("collective_timeout")
    if stall is not None and not ctx.stalled and ctx.rank == (int(stall) if stall else 1):
        ctx.stalled = True
        time.sleep(2 * collective_timeout_s() + 1)
    try:
        if ctx.backend == "nccl":
            # RCCL: the process group's own timeout (watchdog) bounds the call
            dist.all_gather_into_tensor(out, mine)
        else:
            work = dist.all_gather_into_tensor(out, mine, async_op=True)
            work.wait(timeout=timedelta(seconds=collective_timeout_s()))
        host = out.cpu().numpy()
    except Exception as e:  # gloo/RCCL timeout, peer gone, communicator error
        raise CollectiveError(f"rank {ctx.rank}: table all-gather failed: {e}") from e
    tables = []
    for r in range(ctx.world):
        t = brp.CandidateTable()
        t.from_bytes(np.ascontiguousarray(host[r * TABLE_BYTES:(r + 1) * TABLE_BYTES]))
        tables.append(t)
    return tables


def degrade(ctx: DistContext, err: Exception) -> None:
    """Abort this rank's communicators and continue as a single-GPU search."""
    print(f"[brp] WARNING: {err}; aborting the process group and continuing single-GPU", file=sys.stderr,
          flush=True)
    ctx.degraded = True
    try:
        import torch.distributed as dist
        from torch.distributed import distributed_c10d as c10d

        if hasattr(c10d, "_abort_process_group"):
            c10d._abort_process_group()
        else:
            dist.destroy_process_group()
    except Exception as e2:  # already torn down
        print(f"[brp] process group teardown: {e2}", file=sys.stderr, flush=True)


def sharded_merge(run_shard, total: int, ctx: DistContext) -> list:
    """Search `total` templates split over the ranks and merge the tables.

    run_shard(begin, end) returns one candidate table per work unit. If the
    all-gather fails the rank degrades (see `degrade`) and runs the missing
    shards itself, so the merged tables are the same either way."""
    if ctx.solo_shard:
        return run_shard(*shard_range(total, ctx.rank, ctx.world))
    if not ctx.distributed:
        return run_shard(0, total)
    shards = [shard_range(total, r, ctx.world) for r in range(ctx.world)]
    mine = run_shard(*shards[ctx.rank])
    try:
        gathered = [allgather_tables(t, ctx) for t in mine]
    except CollectiveError as e:
        degrade(ctx, e)
        per_rank = [mine if r == ctx.rank else run_shard(*shards[r]) for r in range(len(shards))]
        gathered = [[per_rank[r][w] for r in range(len(shards))] for w in range(len(mine))]
    return [merge_tables(g) for g in gathered]


def merge_tables(tables) -> object:
    """Merge per-shard tables given in template-range order."""
    brp = native()
    out = brp.CandidateTable()
    for t in tables:
        out.merge(t)
    return out


def table_floors(table) -> list[float]:
    """Per harmonic level the power of the 100th entry (0 while the level is
    not full): what a new candidate must beat (demod_binary.c:1281)."""
    ent = table.entries()
    return [float(ent[h * 100 + 99][1]) if ent[h * 100 + 99][5] > 0 else 0.0 for h in range(5)]


def max_floors_over_ranks(floors: list[float], ctx: DistContext) -> list[float]:
    """Element-wise max of the five level floors over the ranks (one 40-byte
    all-reduce): a valid global floor, since every rank's 100 entries of a
    level are distinct bins the merged table also holds at >= that power."""
    if not ctx.distributed:
        return list(floors)
    import torch
    import torch.distributed as dist

    t = torch.tensor(floors, dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu().tolist()]


def floor_sync_interval_s() -> float:
    """Seconds between floor exchanges while a shard runs (BRP_FLOOR_SYNC_MS,
    default 5; 0 disables the exchange)."""
    return float(os.environ.get("BRP_FLOOR_SYNC_MS", "5")) / 1e3


class FloorSync:
    """Global pruning while every rank searches its shard.

    A helper thread all-reduces (max) the five level floors of this rank's
    running table, together with a "still running" flag, over a gloo side
    group, and raises the session's external floors with the result: the
    device thresholds of every rank become the largest 100th-place power any
    rank has reached (demod_binary.c:1268-1282 semantics). That is a valid lower
    bound of the merged table's floor (every rank's 100 entries of a level are
    distinct bins the merge also holds at >= that power), so the filtered bins
    can never enter the merged table. Ranks keep exchanging until the flag is
    clear on all of them, so every rank makes the same number of calls and
    they all leave the loop on the same round."""

    def __init__(self, session, ctx: DistContext, group, interval_s: float):
        self.session, self.ctx, self.group, self.interval = session, ctx, group, interval_s
        self.running = True
        self.rounds = 0
        self.error: Exception | None = None
        self.thread = None

    def start(self) -> "FloorSync":
        import threading

        self.thread = threading.Thread(target=self._loop, name="brp-floor-sync", daemon=True)
        self.thread.start()
        return self

    def _loop(self) -> None:
        import torch
        import torch.distributed as dist

        try:
            while True:
                f = list(self.session.local_floors())
                t = torch.tensor(f + [1.0 if self.running else 0.0], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                self.rounds += 1
                self.session.raise_external_floors([float(v) for v in t[:5].tolist()])
                if t[5].item() == 0.0:
                    return
                time.sleep(self.interval)
        except Exception as e:  # peer gone / timeout: the table all-gather reports it
            self.error = e

    def finish(self) -> None:
        self.running = False
        if self.thread is not None:
            self.thread.join()


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
        self.floor_interval = floor_sync_interval_s()
        self.floor_group = None
        self.floor_rounds = 0  # exchanges of the last step (tests, bench JSON)
        if ctx.distributed and self.floor_interval > 0:
            import torch.distributed as dist

            # CPU side group: the exchange never queues RCCL kernels beside the search
            self.floor_group = dist.new_group(backend="gloo", timeout=timedelta(seconds=collective_timeout_s()))

    def step(self, limit: int | None = None):
        """Whiten + search this rank's shard (exchanging level floors with the
        other ranks while it runs) + all-gather + merge. Returns the merged table."""
        total = self.total if limit is None else min(limit, self.total)
        t0 = time.perf_counter()
        self.session.reset_external_floors()  # every step is an independent search
        self.session.prepare()
        t1 = time.perf_counter()
        search_s = [0.0]

        def run_shard(begin, end):
            ts = time.perf_counter()
            sync = None
            if self.floor_group is not None and self.ctx.distributed:
                sync = FloorSync(self.session, self.ctx, self.floor_group, self.floor_interval).start()
            try:
                table, _ = self.session.run(begin, end, self.brp.CandidateTable())
            finally:
                if sync is not None:
                    sync.finish()
                    self.floor_rounds = sync.rounds
            search_s[0] += time.perf_counter() - ts
            return [table]

        merged = sharded_merge(run_shard, total, self.ctx)[0]
        t3 = time.perf_counter()
        for k, v in (("prepare", t1 - t0), ("templates", search_s[0]), ("merge", t3 - t1 - search_s[0])):
            self.timings[k] = self.timings.get(k, 0.0) + v
        return merged

    def search(self, chunk: int = 2048, kill_after: int | None = None, on_chunk=None):
        """The whole work unit with the application's checkpoint semantics.

        The bank is cut into chunks of `chunk` templates; every rank searches
        its shard_range of the chunk, the tables are all-gathered and merged
        into the running table in template order, so after each chunk the
        merged table covers exactly the prefix [0, n). Rank 0
        then writes the reference-format checkpoint (n, table) atomically.
        A restart reads it on every rank (same node, same file) and resumes at
        n; the result file is written by rank 0 at the end. `kill_after`
        stops (like a BOINC quit: no final checkpoint, no result) after the
        chunk that reaches that many templates. Returns (table, n_done)."""
        brp = self.brp
        cp = self.options.get("checkpointfile") or ""
        table = brp.CandidateTable()
        n = 0
        if cp and os.path.exists(cp):
            got = brp.read_checkpoint(cp)
            if got is not None:
                n_cp, orig, t = got
                if orig != self.options["inputfile"]:
                    raise RuntimeError(f"checkpoint {cp} belongs to {orig}, not {self.options['inputfile']}")
                if n_cp > self.total:
                    raise RuntimeError(f"checkpoint {cp}: {n_cp} templates done > bank size {self.total}")
                n, table = int(n_cp), t
        t0 = time.perf_counter()
        # No FloorSync runs here (each chunk is seeded with the merged prefix
        # table instead): floors a previous step() left behind must not prune
        # this search, or a bin whose power equals one of them is dropped on
        # its own rank and the level ends short of 100 entries.
        self.session.reset_external_floors()
        self.session.prepare()
        t1 = time.perf_counter()
        search_s = 0.0
        self.seed_floors = []  # per chunk: the level floors every rank started from (tests)
        while n < self.total:
            hi = min(self.total, n + max(1, chunk))
            # Global pruning: every rank starts its part of the chunk from the
            # merged table of the prefix, identical on all ranks after the
            # all-gather, so its device and host thresholds are the global
            # 100th-place floors (demod_binary.c:1268-1282 semantics), not those
            # of its own emptier table. Re-merging the seeded entries is exact:
            # the merge keeps one entry per bin and the same entry wins.
            seed = table.to_bytes()
            self.seed_floors.append(table_floors(table))

            def run_shard(begin, end, lo=n, seed=seed):
                nonlocal search_s
                ts = time.perf_counter()
                start = brp.CandidateTable()
                start.from_bytes(np.asarray(seed, dtype=np.uint8).copy())
                t, _ = self.session.run(lo + begin, lo + end, start)
                search_s += time.perf_counter() - ts
                return [t]

            part = sharded_merge(run_shard, hi - n, self.ctx)[0]
            table.merge(part)
            n = hi
            if cp and self.ctx.rank == 0:
                brp.write_checkpoint(cp, n, self.options["inputfile"], table)
            if on_chunk is not None:
                on_chunk(n, self.total)
            if kill_after is not None and n >= kill_after and n < self.total:
                return table, n
        t2 = time.perf_counter()
        for k, v in (("prepare", t1 - t0), ("templates", search_s), ("merge", t2 - t1 - search_s)):
            self.timings[k] = self.timings.get(k, 0.0) + v
        self.write_output(table, n)
        return table, n

    def write_output(self, table, n_done: int | None = None):
        """Rank 0 writes the checkpoint/result files of the merged table."""
        if self.ctx.rank != 0:
            return
        self.brp.finalize_output(self.options, self.session.geometry(),
                                 self.total if n_done is None else n_done, table)
