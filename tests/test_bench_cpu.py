"""The driver-facing bench.py contract on CPU: launched by torch.distributed.run
with 2, 4 and 8 ranks (8: the driver's N=8 shape) (gloo, CPU golden backend, small synthetic WU via --cpu),
rank 0 prints exactly one JSON line with the whole-job value, and the sharded,
all-gathered result file equals the single-rank one byte for byte."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(nproc, tmp, out):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(nproc),
           "--steps", "1", "--warmup", "1", "--cpu", "--batch", "3", "--write-output", str(out)]
    env = dict(os.environ, TMPDIR=str(tmp), OMP_NUM_THREADS="1", BRP_NO_RESULT_HEADER="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_multirank_cpu_rehearsal(nproc, tmp_path):
    one = _bench(1, tmp_path / "w1", tmp_path / "one.cand")
    many = _bench(nproc, tmp_path / f"w{nproc}", tmp_path / "many.cand")
    assert one["n_gpus"] == 1 and many["n_gpus"] == nproc
    assert many["value"] > 0 and many["config"]["parallelism"].startswith(f"dp{nproc}")
    assert many["table_identical_to_warmup"] is True
    assert (tmp_path / "one.cand").read_text() == (tmp_path / "many.cand").read_text()


def _bench_direct(nproc, tmp, out, extra=()):
    """bench.py started WITHOUT a launcher: it must start the ranks itself."""
    cmd = [sys.executable, "bench.py", "--gpus", str(nproc), "--steps", "1", "--warmup", "1", "--cpu", "--batch", "3",
           "--write-output", str(out), *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TMPDIR=str(tmp), OMP_NUM_THREADS="1", BRP_NO_RESULT_HEADER="1")
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)


def test_bench_gpus_without_launcher_starts_the_ranks(tmp_path):
    """`bench.py --gpus 2` with no torchrun: two rank processes, n_gpus 2 in the
    JSON line, the result file equal to the one-rank run byte for byte."""
    one = _bench(1, tmp_path / "w1", tmp_path / "one.cand")
    r = _bench_direct(2, tmp_path / "w2", tmp_path / "two.cand")
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["launched_by"] == "bench.py", rec
    assert rec["floor_sync_rounds_last_step"] >= 1, rec
    assert one["n_gpus"] == 1
    assert (tmp_path / "one.cand").read_text() == (tmp_path / "two.cand").read_text()


def test_bench_world_size_mismatch_is_an_error(tmp_path):
    """A launcher that starts fewer ranks than --gpus asks for is refused
    (the JSON line would otherwise claim a different GPU count)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "WORLD_SIZE=1" in r.stderr


def test_collective_timeout_degrades_to_single_gpu(tmp_path):
    """BRP_FAULT=collective_timeout:1 stalls rank 1 before the all-gather; rank 0
    times out, aborts the process group, searches the missing shard itself and
    writes the same result file as an undisturbed run."""
    one = _bench(1, tmp_path / "w1", tmp_path / "one.cand")
    os.environ["BRP_FAULT"], os.environ["BRP_COLLECTIVE_TIMEOUT"] = "collective_timeout:1", "3"
    try:
        two = _bench(2, tmp_path / "w2", tmp_path / "two.cand")
    finally:
        del os.environ["BRP_FAULT"], os.environ["BRP_COLLECTIVE_TIMEOUT"]
    assert one["collective_failure_degraded"] is False
    assert two["collective_failure_degraded"] is True
    assert (tmp_path / "one.cand").read_text() == (tmp_path / "two.cand").read_text()


def _fake_topology(root: Path, gfx_versions, unreadable=()):
    """KFD topology nodes (gfx_target_version 0 = CPU node) with render nodes."""
    topo, dri = root / "nodes", root / "dri"
    dri.mkdir(parents=True)
    for i, v in enumerate(gfx_versions):
        (topo / str(i)).mkdir(parents=True)
        minor = 128 + i
        (topo / str(i) / "properties").write_text(
            f"cpu_cores_count {0 if v else 64}\ngfx_target_version {v}\ndrm_render_minor {minor if v else 0}\n")
        if v:
            f = dri / f"renderD{minor}"
            f.write_text("")
            f.chmod(0o000 if i in unreadable else 0o666)
    return str(topo), str(dri)


def test_visible_gpus_counts_from_sysfs(tmp_path, monkeypatch):
    """bench.py counts devices without any HIP call (the parent of the rank
    processes must not create a HIP context): GPU nodes of the KFD topology,
    narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES like the runtime."""
    sys.path.insert(0, str(ROOT))
    import bench

    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    topo, dri = _fake_topology(tmp_path / "a", [0, 0, 90500, 90500, 90500, 90500])
    assert bench.visible_gpus(topo, dri) == 4
    assert bench.visible_gpus(str(tmp_path / "missing"), dri) == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,3")
    assert bench.visible_gpus(topo, dri) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,7,1")  # the list ends at the invalid ordinal 7
    assert bench.visible_gpus(topo, dri) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus(topo, dri) == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2")
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "0")
    assert bench.visible_gpus(topo, dri) == 1
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES")
    if os.geteuid() != 0:  # root ignores file modes
        topo2, dri2 = _fake_topology(tmp_path / "b", [0, 90500, 90500], unreadable=(2,))
        assert bench.visible_gpus(topo2, dri2) == 1
