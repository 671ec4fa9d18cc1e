"""Two ranks over RCCL on two MI355X devices (pytest -m gpu; skipped on a
one-GPU box): the sharded search with the all-gathered, rank-ordered merge
equals the one-process table byte for byte, and the chunked search seeds each
rank with the global floors (parallel/dist.py). On a one-GPU box two ranks
share device 0 over gloo instead: the same multi-process path (GPU engines in
two processes, floor exchange during the step, all-gather, merge) without RCCL."""
import os
import socket

import numpy as np
import pytest

from boinc_app_eah_brp_amd.parallel import dist as pdist
from boinc_app_eah_brp_amd.utils import synth

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, opts, out_dir, backend="nccl"):
    # gloo: the ranks share device 0 (LOCAL_RANK 0 selects the engines' GPU)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank if backend == "nccl" else 0),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    ctx = pdist.init_distributed(backend)  # RCCL: the device is set per LOCAL_RANK first
    try:
        assert ctx.backend == backend
        ss = pdist.ShardedSearch(opts, ctx, streams=2)
        table = ss.step()
        chunked, n = ss.search(chunk=9)
        assert n == ss.total
        assert bytes(chunked.to_bytes()) == bytes(table.to_bytes())
        if rank == 0:
            np.save(os.path.join(out_dir, "merged.npy"), np.asarray(table.to_bytes(), np.uint8))
    finally:
        dist.destroy_process_group()


def test_bench_refuses_more_gpus_than_visible(gpu, tmp_path):
    """`bench.py --gpus N` without a launcher starts N ranks itself; asking for
    more GPUs than the box has exits non-zero before any GPU work, with no JSON
    line (it never reports a 1-GPU number as N GPUs)."""
    import subprocess
    import sys

    import torch

    from conftest import ROOT

    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "device(s) are visible" in r.stderr, r.stderr[-2000:]


def test_rccl_two_ranks_equal_single(brp, gpu, tmp_path):
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two HIP devices (the driver's multi-GPU node runs it)")
    import torch.multiprocessing as mp

    inj = synth.Injection(f0=173.0, P_orb=1200.0, tau=0.05, psi0=2.0, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "case", n=1 << 16, n_templates=29, inj=inj)
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=3.0,
                fA=0.08, window=100, white=True, batch=2)
    mp.start_processes(_worker, args=(2, _free_port(), opts, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    merged = np.load(tmp_path / "merged.npy")
    r = brp.run_search(dict(opts), 0, 0, False, False)
    assert r["templates_run"] == 30
    assert bytes(np.asarray(r["table"].to_bytes(), np.uint8)) == bytes(merged)


def test_two_ranks_sharing_one_gpu_gloo(brp, gpu, tmp_path):
    """Two rank processes on device 0 over gloo: GPU engines in each process,
    the level floors exchanged during the step, the all-gathered rank-ordered
    merge equal to the one-process table byte for byte."""
    import torch.multiprocessing as mp

    inj = synth.Injection(f0=173.0, P_orb=1200.0, tau=0.05, psi0=2.0, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "case", n=1 << 16, n_templates=29, inj=inj)
    opts = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=3.0,
                fA=0.08, window=100, white=True, batch=2)
    mp.start_processes(_worker, args=(2, _free_port(), opts, str(tmp_path), "gloo"), nprocs=2, join=True,
                       start_method="spawn")
    merged = np.load(tmp_path / "merged.npy")
    r = brp.run_search(dict(opts), 0, 0, False, False)
    assert r["templates_run"] == 30
    assert bytes(np.asarray(r["table"].to_bytes(), np.uint8)) == bytes(merged)


def test_visible_gpus_matches_the_runtime(gpu):
    """bench.py's HIP-free device count (sysfs) agrees with the runtime's."""
    import sys

    import torch

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import bench

    assert bench.visible_gpus() == torch.cuda.device_count()


def _bench_json(args, env_extra, tmp):
    import json
    import subprocess
    import sys

    from conftest import ROOT

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TMPDIR=str(tmp), BRP_NO_RESULT_HEADER="1", **env_extra)
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_bench_self_launched_ranks_on_one_gpu(gpu, tmp_path, nranks):
    """`bench.py --gpus N` through its own launcher (launch_ranks: N Popen'd
    rank processes, the floor exchange during the step, the all-gather and the
    merge) with BRP_BENCH_SHARE_DEVICE=1, so that all ranks run on this box's
    one GPU over gloo: the table equals the one-rank run's byte for byte. With
    4 and 8 ranks FloorSync's all-reduce has more than two members; 8 is the
    driver's 8-GPU shape (whose first run is otherwise its first execution at
    that size). No throughput is taken from it (the JSON line says so)."""
    common = ["--templates", "200", "--steps", "1", "--warmup", "1"]
    one = _bench_json(["--gpus", "1", *common, "--write-output", str(tmp_path / "one.cand")], {}, tmp_path)
    many = _bench_json(["--gpus", str(nranks), *common, "--write-output", str(tmp_path / "many.cand")],
                       {"BRP_BENCH_SHARE_DEVICE": "1"}, tmp_path)
    assert many["n_gpus"] == nranks and many["launched_by"] == "bench.py", many
    assert "shared_device" in many and "shared_device" not in one
    assert many["floor_sync_rounds_last_step"] > 0, many
    assert many["table_sha256"] == one["table_sha256"]
    assert many["table_identical_to_warmup"] is True
    assert (tmp_path / "one.cand").read_text() == (tmp_path / "many.cand").read_text()
