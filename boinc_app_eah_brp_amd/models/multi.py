"""Multi-work-unit batched search.

The reference runs the work units of one BOINC task as sequential passes
(erp_boinc_wrapper.cpp:411-474). `MultiWUSearch` keeps K same-shape work units
resident in HBM and mixes their templates in every device batch
(csrc/app/multi.cpp); each WU's candidate table still evolves in template
order, exactly as a single-WU run. With torch.distributed, ranks split the
template bank and the K tables are all-gathered and merged per WU.
"""
from __future__ import annotations

import time
from dataclasses import asdict

import numpy as np

from .. import native
from .search import SearchConfig


class MultiWUSearch:
    def __init__(self, inputs: list[str], config: SearchConfig, pipelines: int = 2, device: int = 0, ctx=None):
        from ..parallel.dist import DistContext

        self.brp = native()
        self.inputs = [str(p) for p in inputs]
        self.config = config
        self.ctx = ctx if ctx is not None else DistContext()
        self.session = self.brp.MultiSession()
        dev = self.ctx.local_rank if ctx is not None else device
        self.session.open(self.inputs, asdict(config), max(1, pipelines), [dev] * max(1, pipelines))
        self.total = self.session.total()
        self.timings: dict = {}

    def step(self, limit: int | None = None, block_batches: int = 0):
        """Whiten every WU, search this rank's share of the bank for all WUs,
        all-gather and merge. Returns one candidate table per WU.
        `block_batches` overrides the WU-major deal block (batches per block)."""
        from ..parallel.dist import sharded_merge

        total = self.total if limit is None else min(limit, self.total)
        t0 = time.perf_counter()
        self.session.prepare()
        t1 = time.perf_counter()
        search_s = [0.0]

        def run_shard(begin, end):
            ts = time.perf_counter()
            tables, _ = self.session.run(begin, end, block_batches)
            search_s[0] += time.perf_counter() - ts
            return tables

        merged = sharded_merge(run_shard, total, self.ctx)
        t3 = time.perf_counter()
        for k, v in (("prepare", t1 - t0), ("templates", search_s[0]), ("merge", t3 - t1 - search_s[0])):
            self.timings[k] = self.timings.get(k, 0.0) + v
        return merged

    def write_outputs(self, outputs: list[str], tables, n_done: int | None = None):
        if self.ctx.rank != 0:
            return
        self.session.finalize([str(o) for o in outputs], self.total if n_done is None else n_done, tables)

    def stats(self) -> dict:
        return self.session.stats()


def same_shape_synthetic_wus(workdir, like_header: dict, count: int, seed: int = 100) -> list[str]:
    """`count` synthetic 4-bit WUs with the header geometry of `like_header`
    (noise + one injected binary pulsar each)."""
    from pathlib import Path

    from ..utils import synth

    workdir = Path(workdir)
    workdir.mkdir(parents=True, exist_ok=True)
    out = []
    rng = np.random.default_rng(seed)
    for k in range(count):
        p = workdir / f"synth_{k:03d}.bin4"
        if not p.exists():
            inj = synth.Injection(f0=float(rng.uniform(50, 390)), P_orb=float(rng.uniform(700, 2200)),
                                  tau=float(rng.uniform(0, 0.3)), psi0=float(rng.uniform(0, 6.28)), amplitude=0.3)
            x = synth.make_series(int(like_header["nsamples"]), float(like_header["tsample"]), inj, seed=seed + k)
            synth.write_wu(p, x, float(like_header["tsample"]), name=f"SYNTH{k:03d}")
        out.append(str(p))
    return out
