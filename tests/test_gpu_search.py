"""End-to-end searches on the MI355X against the CPU golden model
(pytest -m gpu). The HIP path must be the one that runs: HipEngine raises if
the device or the extension is missing, there is no silent fallback."""
import os
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth

from conftest import BANK, WU, ZAP

pytestmark = pytest.mark.gpu

INJ = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    return synth.synthetic_case(tmp_path_factory.mktemp("gcase"), n=1 << 16, n_templates=37, inj=INJ)


def _cfg(case, d, **kw):
    d = Path(d)
    d.mkdir(parents=True, exist_ok=True)
    base = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"],
                outputfile=str(d / "out.cand"), checkpointfile=str(d / "cp.cpt"), f0=400.0, padding=3.0, fA=0.08,
                window=100, white=True, batch=4)
    base.update(kw)
    return SearchConfig(**base)


def _entries(table):
    return [e for e in table.entries() if e[5] > 0]


def _compare_tables(t_gpu, t_cpu, rtol=2e-4, margin=1e-4):
    """Same candidate bins per level, both ways, for every entry whose power is
    more than `margin` (relative) above the level's weakest kept power (the
    100th power of a full level); powers within float-FFT tolerance. Only
    entries within `margin` of that boundary may differ (near-ties)."""
    eg, ec = t_gpu.entries(), t_cpu.entries()
    for h in range(5):
        g = {e[0]: e for e in eg[h * 100:(h + 1) * 100] if e[5] > 0}
        c = {e[0]: e for e in ec[h * 100:(h + 1) * 100] if e[5] > 0}
        if not c:  # nothing above the chi^2 threshold on this level
            assert not g, (h, list(g.values())[:3])
            continue
        floor = min(e[1] for e in c.values()) * (1.0 + margin)
        floor_g = min(e[1] for e in g.values()) * (1.0 + margin) if g else 0.0
        for e in c.values():
            if e[1] > floor:
                assert e[0] in g, (h, e)
                assert g[e[0]][1] == pytest.approx(e[1], rel=rtol), (h, e, g[e[0]])
        for e in g.values():
            if e[1] > max(floor, floor_g):
                assert e[0] in c, (h, e)
        assert abs(len(g) - len(c)) <= sum(1 for e in c.values() if e[1] <= floor) + 1


@pytest.mark.parametrize("n,padding", [(1 << 15, 1.0), (1 << 16, 2.0), (3 << 14, 3.0), (5 << 14, 1.0)])
def test_fft_plans_power_spectrum(brp, gpu, tmp_path, n, padding):
    """Different FFT factorisations (L1 x L2 x L3) against the double CPU FFT."""
    x = synth.make_series(n, 65.476, synth.Injection(f0=97.0, P_orb=700.0, tau=0.02, psi0=0.3, amplitude=2.0))
    wu = synth.write_wu(tmp_path / "a.bin4", x)
    hdr, series, _ = brp.read_work_unit(str(wu))
    geom = brp.derive_geometry(hdr, dict(f0=150.0, padding=padding, fA=0.08, window=100))
    M = geom["nsamples"] // 2
    assert brp.fft_plan(M) is not None, M
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, series, float(np.mean(series)))
    for P, tau, psi in ((700.0, 0.02, 0.3), (1500.0, 0.3, 4.0)):
        ps_g, ns_g = eng.power_spectrum(P, tau, psi)
        xr, ns_c, _ = brp.cpu_resample(series, geom, P, tau, psi)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        assert ns_g == ns_c
        scale = float(np.mean(ps_c[1:]))
        err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
        assert err.max() < 2e-4, (n, padding, err.max())


def test_gpu_search_matches_cpu(brp, gpu, case, tmp_path):
    g = BRPSearch(_cfg(case, tmp_path / "g")).run()
    c = BRPSearch(_cfg(case, tmp_path / "c", use_cpu=True)).run()
    assert g.templates_run == c.templates_run == 38
    _compare_tables(g.table, c.table)
    lg, _ = brp.read_results(str(tmp_path / "g" / "out.cand"))
    lc, _ = brp.read_results(str(tmp_path / "c" / "out.cand"))
    # the top result lines (strongest candidates) agree
    for a, b in zip(lg[:10], lc[:10]):
        assert a[0] == pytest.approx(b[0], rel=1e-9) and a[6] == b[6]
        assert a[4] == pytest.approx(b[4], rel=2e-4)


def test_gpu_block_runs_merge_to_full(brp, gpu, case, tmp_path):
    full = BRPSearch(_cfg(case, tmp_path / "f")).run(write_output=False, use_checkpoint=False)
    merged = brp.CandidateTable()
    for b, e in ((0, 9), (9, 10), (10, 38)):
        o = BRPSearch(_cfg(case, tmp_path / "p", batch=3)).run(begin=b, end=e, write_output=False,
                                                               use_checkpoint=False)
        merged.merge(o.table)
    _compare_tables(merged, full.table, rtol=1e-6)


def test_two_backends_one_process(brp, gpu, case, tmp_path):
    """Two device backends fed by worker threads, applied in template order
    (the in-process multi-GPU path; both on device 0 on a one-GPU box)."""
    opts = _cfg(case, tmp_path / "m").options()
    s = brp.SearchSession()
    s.open(opts, 2, [0, 0])
    s.prepare()
    t2, _ = s.run(0, s.total(), brp.CandidateTable())
    one = BRPSearch(_cfg(case, tmp_path / "o")).run(write_output=False, use_checkpoint=False)
    assert bytes(t2.to_bytes()) == bytes(one.table.to_bytes())


def test_bench_wu_prefix_vs_cpu_golden(brp, gpu, tmp_path):
    """First templates of the benchmark WU (whitened, 3*2^22-point FFT) on the GPU
    vs the CPU golden model."""
    kw = dict(batch=4)
    cfg = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), outputfile=str(tmp_path / "g.cand"), **kw)
    g = BRPSearch(cfg).run(begin=0, end=12, write_output=False, use_checkpoint=False)
    cfgc = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), outputfile=str(tmp_path / "c.cand"), batch=1,
                                  use_cpu=True)
    c = BRPSearch(cfgc, gpus=12).run(begin=0, end=12, write_output=False, use_checkpoint=False)
    _compare_tables(g.table, c.table)


def test_app_binary_gpu(brp, gpu, case, tmp_path):
    app = app_binary()
    assert app.exists()
    args = ["-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o", str(tmp_path / "res.cand"), "-c",
            str(tmp_path / "cp.cpt"), "-A", "0.08", "-P", "3.0", "-f", "400.0", "-W", "-B", "100"]
    env = dict(os.environ, BRP_NO_RESULT_HEADER="1")
    r = subprocess.run([str(app), *args], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines, done = brp.read_results(str(tmp_path / "res.cand"))
    assert done and lines
    rc = BRPSearch(_cfg(case, tmp_path / "c", use_cpu=True)).run()
    lc, _ = brp.read_results(str(tmp_path / "c" / "out.cand"))
    assert lines[0][0] == pytest.approx(lc[0][0], rel=1e-9)


@pytest.mark.parametrize("block_batches", [0, 1, 2])
def test_multi_wu_batching_matches_single_runs(brp, gpu, tmp_path, block_batches):
    """K same-shape WUs resident together, dealt WU-major in blocks of
    block_batches batches (0 = default 64: one block holds the 21-template bank;
    1 and 2 cross many block boundaries): each WU's table equals its own
    single-WU run byte for byte."""
    from boinc_app_eah_brp_amd.models import MultiWUSearch

    wus = []
    for k in range(3):
        inj = synth.Injection(f0=150.0 + 40 * k, P_orb=900.0 + 100 * k, tau=0.02, psi0=0.5 * k, amplitude=3.0)
        c = synth.synthetic_case(tmp_path / f"w{k}", n=1 << 16, n_templates=21, inj=inj, seed=10 + k)
        wus.append(c)
    bank = wus[0]["bank"]
    cfg = SearchConfig(inputfile=wus[0]["wu"], templatebank=bank, zaplistfile=wus[0]["zap"], f0=400.0, padding=3.0,
                       fA=0.08, window=100, white=True, batch=4)
    ms = MultiWUSearch([c["wu"] for c in wus], cfg, pipelines=2)
    tables = ms.step(block_batches=block_batches)
    assert len(tables) == 3
    for k, c in enumerate(wus):
        single = BRPSearch(_cfg(c, tmp_path / f"s{k}", templatebank=bank, batch=4)).run(write_output=False,
                                                                                      use_checkpoint=False)
        assert bytes(tables[k].to_bytes()) == bytes(single.table.to_bytes()), k
    outs = [str(tmp_path / f"o{k}.cand") for k in range(3)]
    ms.write_outputs(outs, tables)
    for o in outs:
        lines, done = brp.read_results(o)
        assert done and lines


def test_fp16_power_spectrum_config(brp, gpu, case, tmp_path):
    """Config 5: fp16 spectrum between pass 3 and the harmonic sum. The strong
    candidates are the fp32 ones (same bins), powers within fp16 rounding."""
    f32 = BRPSearch(_cfg(case, tmp_path / "a")).run(write_output=False, use_checkpoint=False)
    f16 = BRPSearch(_cfg(case, tmp_path / "b", ps_fp16=True)).run(write_output=False, use_checkpoint=False)
    _compare_tables(f16.table, f32.table, rtol=3e-3)
    with pytest.raises(RuntimeError):
        BRPSearch(_cfg(case, tmp_path / "c", ps_fp16=True, white=False)).run(write_output=False,
                                                                           use_checkpoint=False)


def _app_gpu(case, d, **env):
    d = Path(d)
    d.mkdir(parents=True, exist_ok=True)
    args = ["-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o", str(d / "res.cand"), "-c",
            str(d / "cp.cpt"), "-A", "0.08", "-P", "3.0", "-f", "400.0", "-W", "-B", "100"]
    e = dict(os.environ, BRP_NO_RESULT_HEADER="1", **env)
    return subprocess.run([str(app_binary()), *args], cwd=d, env=e, capture_output=True, text=True, timeout=300)


def test_fault_hip_oom_temporary_exit(brp, gpu, case, tmp_path):
    """Device allocation failure -> BOINC temporary exit, no result written
    (erp_boinc_wrapper.cpp:560-570)."""
    r = _app_gpu(case, tmp_path, BRP_FAULT="hip_oom")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Temporary exit (900 s)" in r.stderr, r.stderr[-3000:]
    assert "device memory" in r.stderr
    assert not (tmp_path / "res.cand").exists()


def test_fault_hip_oom_later_pipeline_temporary_exit(brp, gpu, case, tmp_path):
    """Only the allocations after the first pipeline's setup fail (a later
    pipeline takes the whitened series device to device): still a BOINC
    temporary exit, not a hard error."""
    probe = _app_gpu(case, tmp_path / "probe", BRP_LOGLEVEL="4")
    assert probe.returncode == 0, probe.stderr[-3000:]
    m = re.search(r"HIP device allocations so far: (\d+)", probe.stdout + probe.stderr)
    assert m, (probe.stdout + probe.stderr)[-3000:]
    n_first = int(m.group(1))
    r = _app_gpu(case, tmp_path / "oom", BRP_FAULT=f"hip_oom:{n_first}")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Temporary exit (900 s)" in r.stderr, r.stderr[-3000:]
    assert not (tmp_path / "oom" / "res.cand").exists()


def test_fault_pinned_fail_falls_back_to_pageable(brp, gpu, case, tmp_path):
    """Pinned host allocation failure -> pageable buffers, identical results
    (cuda/app/demod_binary_hs_cuda.cu:207-219)."""
    a = _app_gpu(case, tmp_path / "a", BRP_FG="0")
    b = _app_gpu(case, tmp_path / "b", BRP_FAULT="pinned_fail", BRP_FG="0")
    assert a.returncode == 0 and b.returncode == 0, b.stderr[-3000:]
    assert "pageable" in b.stderr
    assert (tmp_path / "a" / "res.cand").read_bytes() == (tmp_path / "b" / "res.cand").read_bytes()


def test_fine_grained_parameter_and_result_buffers(brp, gpu, case, tmp_path):
    """Batch parameters / candidate lists in host-visible fine-grained device
    memory (BRP_FG, default "in") give the same result file as the copy path."""
    runs = {}
    for fg in ("0", "in", "out", "both"):
        r = _app_gpu(case, tmp_path / fg, BRP_FG=fg, BRP_LOGLEVEL="4")
        assert r.returncode == 0, r.stderr[-3000:]
        assert "not host visible" not in r.stderr, r.stdout[-2000:]
        if fg != "0":
            assert "large BAR 1" in r.stdout + r.stderr
        runs[fg] = (tmp_path / fg / "res.cand").read_bytes()
    assert runs["in"] == runs["0"] and runs["out"] == runs["0"] and runs["both"] == runs["0"]


_RCCL_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from boinc_app_eah_brp_amd import native
from boinc_app_eah_brp_amd.parallel import dist as bd
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
class Forced(bd.DistContext):
    distributed = property(lambda self: True)
ctx = Forced(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
t = native().CandidateTable()
got = bd.allgather_tables(t, ctx)
assert len(got) == 1 and bytes(got[0].to_bytes()) == bytes(t.to_bytes())
assert bd.max_over_ranks(3.5, ctx) == 3.5
bd.barrier(ctx)
dist.destroy_process_group()
print("RCCL_OK")
"""


def test_rccl_collectives_single_rank(gpu, tmp_path):
    """The RCCL calls of the sharded search (uint8 all-gather of the tables,
    float64 max all-reduce, barrier) on a one-rank process group."""
    import socket
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               REPO=str(Path(__file__).resolve().parent.parent))
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, r.stderr[-3000:]


_SHARD_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.environ["REPO"])
import json, numpy as np, torch, torch.distributed as dist
from boinc_app_eah_brp_amd.parallel import dist as bd
opts = json.loads(os.environ["OPTS"])
ctx = bd.init_distributed("gloo")
ss = bd.ShardedSearch(opts, ctx, device=0, streams=2)
table = ss.step()
if ctx.rank == 0:
    np.save(os.environ["OUT"], np.asarray(table.to_bytes(), np.uint8))
bd.barrier(ctx)
dist.destroy_process_group()
print("SHARD_OK", ctx.rank, ss.begin, ss.end)
"""


def test_two_rank_sharded_gpu_search_equals_single(brp, gpu, case, tmp_path):
    """The multi-rank bench path with HIP engines: two ranks (gloo; RCCL
    refuses two ranks on one GPU) each search half the bank on the GPU, the
    all-gathered merge equals a one-rank search byte for byte."""
    import json
    import socket
    import sys

    import numpy as np

    from boinc_app_eah_brp_amd.parallel import dist as bd

    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=3.0,
                fA=0.08, window=100, white=True, batch=2, outputfile=str(tmp_path / "x.cand"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "merged.npy"
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                   LOCAL_RANK="0", OPTS=json.dumps(opts), OUT=str(out),
                   REPO=str(Path(__file__).resolve().parent.parent))
        procs.append(subprocess.Popen([sys.executable, "-c", _SHARD_SCRIPT], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        so, se = p.communicate(timeout=240)
        assert p.returncode == 0 and "SHARD_OK" in so, se[-3000:]

    single = bd.ShardedSearch(opts, bd.DistContext(rank=0, world=1, local_rank=0, backend="none"), device=0,
                              streams=2).step()
    assert bytes(np.load(out)) == bytes(np.asarray(single.to_bytes(), np.uint8))
    assert sum(1 for e in single.entries() if e[5] > 0) > 0


def test_pipelines_sharing_one_series_equal_single_pipeline(brp, gpu, case, tmp_path):
    """Three pipelines on one device: after the first pass, pipelines 2 and 3
    read pipeline 1's whitened series in place (HipEngine::adopt_series). Every
    pass, the shared one included, gives the one-pipeline table byte for byte."""
    from boinc_app_eah_brp_amd.parallel import dist as bd

    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=3.0,
                fA=0.08, window=100, white=True, batch=1, outputfile=str(tmp_path / "x.cand"))
    ctx = bd.DistContext(rank=0, world=1, local_rank=0, backend="none")
    one = bytes(bd.ShardedSearch(opts, ctx, device=0, streams=1).step().to_bytes())
    three = bd.ShardedSearch(opts, ctx, device=0, streams=3)
    shared = []
    for _ in range(3):
        assert bytes(three.step().to_bytes()) == one
        shared.append(three.session.stats()["shared_series_batches"])
    # passes 2 and 3 really read pipeline 1's series in place (not a copy each)
    assert shared[1] > shared[0] and shared[2] > shared[1], shared


def test_peer_series_copy_equals_single_pipeline(brp, gpu, case, tmp_path, monkeypatch):
    """Pipelines on other devices take the whitened series by hipMemcpyPeer
    (no host round trip). One box has one GPU, so BRP_PEER_SERIES=1 forces that
    path between pipelines of device 0: same table as one pipeline, copies
    counted, nothing read in place."""
    from boinc_app_eah_brp_amd.parallel import dist as bd

    monkeypatch.setenv("BRP_PEER_SERIES", "1")
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=3.0,
                fA=0.08, window=100, white=True, batch=1, outputfile=str(tmp_path / "x.cand"))
    ctx = bd.DistContext(rank=0, world=1, local_rank=0, backend="none")
    one = bytes(bd.ShardedSearch(opts, ctx, device=0, streams=1).step().to_bytes())
    three = bd.ShardedSearch(opts, ctx, device=0, streams=3)
    for step in range(2):
        assert bytes(three.step().to_bytes()) == one
        st = three.session.stats()
        assert st["peer_series_copies"] == 2 * (step + 1), st
        assert st["shared_series_batches"] == 0, st


def test_stale_adopted_series_is_refused(brp, gpu, case):
    """A pipeline that adopted another engine's series must not launch once the
    source rewrote it (set up again for another WU) or was destroyed."""
    hdr, series, _ = brp.read_work_unit(case["wu"])
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=3.0, fA=0.08, window=100))
    src, rd = brp.HipEngine(), brp.HipEngine()
    for e in (src, rd):
        e.init(0, 1)
        e.setup(geom, series, float(np.mean(series)))
    P, tau, psi = brp.read_template_bank(case["bank"])
    args = (P[:1].astype(np.float32), tau[:1].astype(np.float32), psi[:1].astype(np.float32), [30.0] * 5)
    rd.adopt_series(src)
    rd.process(*args)  # valid while the source is unchanged
    src.setup(geom, series * 2.0, float(np.mean(series)) * 2.0)  # rewrites the adopted buffer
    with pytest.raises(RuntimeError):
        rd.process(*args)
    rd.adopt_series(src)
    rd.process(*args)
    del src
    import gc
    gc.collect()
    with pytest.raises(RuntimeError):
        rd.process(*args)
