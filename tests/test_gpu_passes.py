"""Batched multi-pass BOINC task (csrc/app/passes.cpp) against the reference's
sequential passes (erp_boinc_wrapper.cpp:411-474): byte-identical result
files, the skip-existing-output rule, per-WU checkpoints with quit + resume."""
import os
import struct
import subprocess
from pathlib import Path

import pytest

from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def task(tmp_path_factory):
    d = tmp_path_factory.mktemp("passes")
    wus = []
    for k in range(3):
        inj = synth.Injection(f0=140.0 + 50 * k, P_orb=800.0 + 150 * k, tau=0.02, psi0=0.4 + k, amplitude=3.0)
        wus.append(synth.synthetic_case(d / f"w{k}", n=1 << 16, n_templates=21, inj=inj, seed=20 + k))
    return dict(wus=[c["wu"] for c in wus], bank=wus[0]["bank"], zap=wus[0]["zap"])


def _args(task, outs, extra=()):
    a = [str(app_binary())]
    for w, o in zip(task["wus"], outs):
        a += ["-i", w, "-o", str(o)]
    return a + ["-t", task["bank"], "-l", task["zap"], "-c", "cp.cpt", "-A", "0.08", "-P", "3.0", "-f", "400.0",
                "-W", "-B", "100", *extra]


def _run(args, cwd, **env):
    return subprocess.run(args, cwd=cwd, capture_output=True, text=True, timeout=300,
                          env=dict(os.environ, BRP_CHECKPOINT_PERIOD="0", **env))


def _body(path):
    # the provenance header carries the date; everything else must match
    return [l for l in Path(path).read_text().splitlines() if not l.startswith("% Date")]


@pytest.fixture(scope="module")
def sequential(task, tmp_path_factory):
    d = tmp_path_factory.mktemp("seq")
    outs = [d / f"o{k}.cand" for k in range(3)]
    r = _run(_args(task, outs, ["--mi355x-sequential-passes"]), d)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "batched pass" not in r.stderr
    return [_body(o) for o in outs]


def test_batched_passes_equal_sequential(gpu, task, sequential, tmp_path):
    outs = [tmp_path / f"o{k}.cand" for k in range(3)]
    r = _run(_args(task, outs), tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "3 work units in one batched pass" in r.stderr
    for k in range(3):
        assert _body(outs[k]) == sequential[k], k
    # checkpoints of finished passes are deleted
    assert not list(tmp_path.glob("cp.cpt*"))
    assert (tmp_path / "boinc_finish_called").read_text().strip() == "0"


def test_batched_passes_skip_existing_output(gpu, task, sequential, tmp_path):
    outs = [tmp_path / f"o{k}.cand" for k in range(3)]
    outs[1].write_text("already here\n")
    r = _run(_args(task, outs), tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "already exists - skipping pass" in r.stderr
    assert "2 work units in one batched pass" in r.stderr
    assert outs[1].read_text() == "already here\n"
    assert _body(outs[0]) == sequential[0] and _body(outs[2]) == sequential[2]


def test_batched_passes_quit_and_resume(gpu, task, sequential, tmp_path):
    outs = [tmp_path / f"o{k}.cand" for k in range(3)]
    # one-template deal blocks: a checkpoint point after every template of all WUs
    env = dict(BRP_MULTI_BLOCK="1")
    r = _run(_args(task, outs, ["--mi355x-pipelines", "2"]), tmp_path, BRP_FAULT="kill_after_template:8", **env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "quit prematurely" in r.stderr
    assert not any(o.exists() for o in outs)
    assert not (tmp_path / "boinc_finish_called").exists()
    done = []
    for k in range(3):
        data = (tmp_path / f"cp.cpt.{k}").read_bytes()
        assert len(data) == 24260
        done.append(struct.unpack("<I", data[:4])[0])
    assert all(8 <= n < 22 for n in done), done
    r = _run(_args(task, outs), tmp_path, **env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stderr.count("Continuing work on") == 3
    for k in range(3):
        assert _body(outs[k]) == sequential[k], k
    assert not list(tmp_path.glob("cp.cpt*"))


def test_batched_passes_resume_from_legacy_checkpoint(gpu, task, sequential, tmp_path):
    """A reference-style checkpoint (one file, the first pass interrupted by the
    sequential wrapper) resumes that WU at its template while the other WUs
    start at 0; with 4-template batches the deal blocks are then no multiple
    of the batch, and batches are cut at block boundaries. Results equal the
    uninterrupted sequential passes byte for byte."""
    outs = [tmp_path / f"o{k}.cand" for k in range(3)]
    r = _run(_args(task, outs, ["--mi355x-sequential-passes"]), tmp_path, BRP_FAULT="kill_after_template:5")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "quit prematurely" in r.stderr
    data = (tmp_path / "cp.cpt").read_bytes()
    n0 = struct.unpack("<I", data[:4])[0]
    assert 5 <= n0 < 22, n0
    env = dict(BRP_MULTI_BLOCK="1")
    # interrupted once more inside the batched pass, then finished
    r = _run(_args(task, outs, ["--mi355x-batch", "4"]), tmp_path, BRP_FAULT="kill_after_template:12", **env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Continuing work on" in r.stderr
    r = _run(_args(task, outs, ["--mi355x-batch", "4"]), tmp_path, **env)
    assert r.returncode == 0, r.stderr[-3000:]
    for k in range(3):
        assert _body(outs[k]) == sequential[k], k
    assert not list(tmp_path.glob("cp.cpt*"))
