"""Template-bank sharding over torch.distributed on CPU (gloo, world_size 2):
the all-gathered, rank-ordered merge must reproduce the single-process table
byte for byte (parallel/dist.py)."""
import os
import socket

import numpy as np
import pytest

from boinc_app_eah_brp_amd.parallel import dist as pdist
from boinc_app_eah_brp_amd.utils import synth


def test_shard_range_partitions():
    for total in (0, 1, 7, 8, 6662):
        for world in (1, 2, 3, 8):
            ranges = [pdist.shard_range(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and b - a >= d - c >= b - a - 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, opts, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    ctx = pdist.init_distributed("gloo")
    try:
        ss = pdist.ShardedSearch(opts, ctx, use_cpu=True)
        table = ss.step()
        m = pdist.max_over_ranks(float(rank + 1), ctx)
        assert m == float(world)
        if rank == 0:
            np.save(os.path.join(out_dir, "merged.npy"), np.asarray(table.to_bytes(), np.uint8))
            ss.write_output(table)
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_equals_single(brp, tmp_path):
    import torch.multiprocessing as mp

    inj = synth.Injection(f0=173.0, P_orb=1200.0, tau=0.05, psi0=2.0, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "case", n=1 << 15, n_templates=19, inj=inj)
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"],
                outputfile=str(tmp_path / "dist.cand"), checkpointfile=str(tmp_path / "dist.cpt"), f0=400.0,
                padding=3.0, fA=0.08, window=100, white=True, batch=3, use_cpu=True)
    mp.start_processes(_worker, args=(2, _free_port(), opts, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    merged = np.load(tmp_path / "merged.npy")

    single = dict(opts, outputfile=str(tmp_path / "single.cand"), checkpointfile=str(tmp_path / "single.cpt"))
    r = brp.run_search(single, 0, 0, True, False)
    assert r["templates_run"] == 20
    assert bytes(np.asarray(r["table"].to_bytes(), np.uint8)) == bytes(merged)
    # identical result files (ignoring the optional comment header)
    strip = lambda p: [l for l in open(p).read().splitlines() if not l.startswith("% ")]
    assert strip(tmp_path / "dist.cand") == strip(tmp_path / "single.cand")
