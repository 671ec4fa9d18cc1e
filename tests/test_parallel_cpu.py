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


def _cp_worker(rank, world, port, opts, out_dir, kill_after):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    ctx = pdist.init_distributed("gloo")
    try:
        ss = pdist.ShardedSearch(opts, ctx, use_cpu=True)
        table, n = ss.search(chunk=7, kill_after=kill_after)
        # every chunk started from the merged prefix: the seeds' floors rise
        # monotonically and equal the max over ranks (identical merged tables)
        for a, b in zip(ss.seed_floors, ss.seed_floors[1:]):
            assert all(y >= x for x, y in zip(a, b)), (a, b)
        mine = pdist.table_floors(table)
        assert pdist.max_floors_over_ranks(mine, ctx) == mine
        if rank == 0:
            np.save(os.path.join(out_dir, f"n_{kill_after}.npy"), np.array([n]))
            np.save(os.path.join(out_dir, f"floors_{kill_after}.npy"), np.array(ss.seed_floors))
    finally:
        dist.destroy_process_group()


def test_gloo_chunked_checkpoint_resume_equals_single(brp, tmp_path):
    """torchrun path with the app's checkpoint semantics: chunks of 7 templates
    all-gathered and merged in order, rank 0 checkpoints the prefix after each
    chunk; a run stopped after 14 templates resumes from the checkpoint on a new
    process group and writes the single-process result file byte for byte."""
    import torch.multiprocessing as mp

    inj = synth.Injection(f0=173.0, P_orb=1200.0, tau=0.05, psi0=2.0, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "case", n=1 << 14, n_templates=29, inj=inj)
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"],
                outputfile=str(tmp_path / "dist.cand"), checkpointfile=str(tmp_path / "dist.cpt"), f0=400.0,
                padding=3.0, fA=0.08, window=100, white=True, batch=2, use_cpu=True)
    os.environ["BRP_NO_RESULT_HEADER"] = "1"
    try:
        mp.start_processes(_cp_worker, args=(2, _free_port(), opts, str(tmp_path), 14), nprocs=2, join=True,
                           start_method="spawn")
        assert int(np.load(tmp_path / "n_14.npy")[0]) == 14
        assert not os.path.exists(opts["outputfile"])
        n_cp, orig, _ = brp.read_checkpoint(opts["checkpointfile"])
        assert n_cp == 14 and orig == case["wu"]
        mp.start_processes(_cp_worker, args=(2, _free_port(), opts, str(tmp_path), None), nprocs=2, join=True,
                           start_method="spawn")
        assert int(np.load(tmp_path / "n_None.npy")[0]) == 30
        assert np.load(tmp_path / "floors_None.npy")[-1].max() > 0  # later chunks prune with a real floor
        single = dict(opts, outputfile=str(tmp_path / "single.cand"), checkpointfile=str(tmp_path / "single.cpt"))
        r = brp.run_search(single, 0, 0, True, False)
        assert r["templates_run"] == 30
    finally:
        del os.environ["BRP_NO_RESULT_HEADER"]
    assert open(opts["outputfile"]).read() == open(single["outputfile"]).read()
    n_cp, _, _ = brp.read_checkpoint(opts["checkpointfile"])
    assert n_cp == 30


def test_external_floors_keep_entries_at_the_floor(brp, tmp_path):
    """Pruning with other ranks' level floors is exact (advisor round 4):
    a rank whose shard holds a level's whole top 100 exchanges floors equal to
    the merged table's; the bins whose power equals a floor must still reach
    the applier (the device emits p > thr, so thr sits just below the floor),
    and search() must not inherit the floors a previous step() left behind."""
    inj = synth.Injection(f0=173.0, P_orb=1200.0, tau=0.05, psi0=2.0, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "case", n=1 << 14, n_templates=11, inj=inj)
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"],
                outputfile=str(tmp_path / "o.cand"), checkpointfile=str(tmp_path / "o.cpt"), f0=400.0,
                padding=3.0, fA=0.999, window=100, white=True, batch=3, use_cpu=True)
    ss = pdist.ShardedSearch(opts, pdist.DistContext(), use_cpu=True)
    ref = bytes(np.asarray(ss.step().to_bytes(), np.uint8))
    t_ref = brp.CandidateTable()
    t_ref.from_bytes(np.frombuffer(ref, np.uint8).copy())
    floors = pdist.table_floors(t_ref)
    assert sum(f > 0 for f in floors) >= 2, floors  # full levels: their 100th entry sits at the floor

    # one rank owning the whole top 100: the exchanged floors equal the merged ones
    ss.session.reset_external_floors()
    ss.session.raise_external_floors(floors)
    t, _ = ss.session.run(0, ss.total, brp.CandidateTable())
    assert bytes(np.asarray(t.to_bytes(), np.uint8)) == ref

    # floors left over from an earlier exchange (here: above every power) must not prune search()
    ss.session.raise_external_floors([3.0e38] * 5)
    table, n = ss.search(chunk=4)
    assert n == ss.total
    assert bytes(np.asarray(table.to_bytes(), np.uint8)) == ref
