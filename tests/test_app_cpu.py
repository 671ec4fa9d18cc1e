"""End-to-end searches on the CPU golden backend: the Python driver, the BOINC
application binary (wrapper + MAIN parser), checkpoint/resume under fault
injection, and the command-line contract (erp_boinc_wrapper.cpp:147-300,
demod_binary.c:117-700)."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth

INJ = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    d = tmp_path_factory.mktemp("case")
    return synth.synthetic_case(d, n=1 << 15, n_templates=23, inj=INJ)


@pytest.fixture(scope="module")
def app(brp):
    p = app_binary()
    if not p.exists():
        from boinc_app_eah_brp_amd import _build

        _build.build()
    assert p.exists()
    return p


def _cfg(case, d, **kw):
    d = Path(d)
    base = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"],
                outputfile=str(d / "out.cand"), checkpointfile=str(d / "cp.cpt"), f0=400.0, padding=3.0, fA=0.08,
                window=100, white=True, batch=4, use_cpu=True)
    base.update(kw)
    return SearchConfig(**base)


def _result_lines(path):
    return [l for l in Path(path).read_text().splitlines() if l and not l.startswith("%") or l == "%DONE%"]


def test_cpu_search_finds_injection(brp, case, tmp_path):
    s = BRPSearch(_cfg(case, tmp_path))
    out = s.run()
    assert out.templates_run == out.templates_total == 24
    lines, done = s.results()
    assert done and lines
    f, P, tau, psi, power, fa, nh = lines[0]
    # the strongest candidate is the injected spin frequency (or a harmonic of it)
    r = f / INJ.f0
    assert abs(r - round(r)) < 0.01 or abs(1 / r - round(1 / r)) < 0.01, lines[:3]
    assert fa > 20


def test_python_driver_block_runs_merge_to_full(brp, case, tmp_path):
    full = BRPSearch(_cfg(case, tmp_path / "a")).run(write_output=False, use_checkpoint=False)
    tables = []
    for b, e in ((0, 7), (7, 8), (8, 24)):
        o = BRPSearch(_cfg(case, tmp_path / "b")).run(begin=b, end=e, write_output=False, use_checkpoint=False)
        tables.append(o.table)
    merged = brp.CandidateTable()
    for t in tables:
        merged.merge(t)
    assert bytes(full.table.to_bytes()) == bytes(merged.to_bytes())


def _app_args(case, d, extra=()):
    d = Path(d)
    return ["-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o", str(d / "res.cand"), "-c",
            str(d / "cp.cpt"), "-A", "0.08", "-P", "3.0", "-f", "400.0", "-W", "-B", "100", "--mi355x-cpu", *extra]


def _run_app(app, args, cwd, **env):
    e = dict(os.environ, BRP_NO_RESULT_HEADER="1", **env)
    return subprocess.run([str(app), *args], cwd=cwd, env=e, capture_output=True, text=True, timeout=300)


def test_app_checkpoint_resume_after_fault(app, case, tmp_path):
    ref_dir, run_dir = tmp_path / "ref", tmp_path / "run"
    ref_dir.mkdir()
    run_dir.mkdir()
    r = _run_app(app, _app_args(case, ref_dir), ref_dir)
    assert r.returncode == 0, r.stderr[-2000:]
    ref = _result_lines(ref_dir / "res.cand")
    assert ref[-1] == "%DONE%"
    # checkpoint file is removed after a successful pass
    assert not (ref_dir / "cp.cpt").exists()

    # interrupted after 9 templates (checkpoint every template), then resumed
    r = _run_app(app, _app_args(case, run_dir), run_dir, BRP_FAULT="kill_after_template:9", BRP_CHECKPOINT_PERIOD="0")
    assert r.returncode == 0, r.stderr[-2000:]
    assert not (run_dir / "res.cand").exists()
    assert (run_dir / "cp.cpt").exists()
    import boinc_app_eah_brp_amd as pkg

    n, orig, _ = pkg.native().read_checkpoint(str(run_dir / "cp.cpt"))
    assert 9 <= n < 24 and orig == case["wu"]
    r = _run_app(app, _app_args(case, run_dir), run_dir)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Continuing work on" in r.stderr or "checkpoint" in r.stderr.lower()
    assert _result_lines(run_dir / "res.cand") == ref


def test_app_skips_existing_output(app, case, tmp_path):
    (tmp_path / "res.cand").write_text("keep\n")
    r = _run_app(app, _app_args(case, tmp_path), tmp_path)
    assert r.returncode == 0
    assert "already exists" in r.stderr
    assert (tmp_path / "res.cand").read_text() == "keep\n"


def test_app_rejects_checkpoint_of_other_input(app, brp, case, tmp_path):
    brp.write_checkpoint(str(tmp_path / "cp.cpt"), 3, "some_other_file.bin4", brp.CandidateTable())
    r = _run_app(app, _app_args(case, tmp_path), tmp_path)
    assert r.returncode != 0
    assert "doesn't agree" in r.stderr


def test_app_option_errors(app, case, tmp_path):
    # -K (kill line) is accepted by the wrapper but rejected by MAIN (reference quirk)
    r = _run_app(app, _app_args(case, tmp_path, ["-K"]), tmp_path)
    assert r.returncode != 0
    # unequal numbers of -i and -o
    r = _run_app(app, ["-i", case["wu"], "-t", case["bank"]], tmp_path)
    assert r.returncode != 0
    r = _run_app(app, ["--version"], tmp_path)
    assert r.returncode == 0 and "Binary Pulsar Search Revision" in r.stderr + r.stdout


def test_app_soft_link_resolution(app, case, tmp_path):
    # BOINC logical names: a file containing <soft_link>physical</soft_link>
    (tmp_path / "logical_wu").write_text(f"<soft_link>{case['wu']}</soft_link>\n")
    args = _app_args(case, tmp_path)
    args[1] = "logical_wu"
    # the checkpoint header holds the physical file name
    r = _run_app(app, args, tmp_path, BRP_FAULT="kill_after_template:2", BRP_CHECKPOINT_PERIOD="0")
    assert r.returncode == 0, r.stderr[-2000:]
    import boinc_app_eah_brp_amd as pkg

    _, orig, _ = pkg.native().read_checkpoint(str(tmp_path / "cp.cpt"))
    assert orig == case["wu"]


def test_search_main_in_process(brp, case, tmp_path):
    rc = BRPSearch.command_line(["prog", *_app_args(case, tmp_path)])
    assert rc == 0
    lines, done = brp.read_results(str(tmp_path / "res.cand"))
    assert done and len(lines) > 0
    # invalid option value
    assert BRPSearch.command_line(["prog", "-P", "0.5", *_app_args(case, tmp_path)[0:4]]) != 0


def test_shmem_xml_render(brp):
    xml = brp.render_shmem_xml()
    # element names of erp_boinc_ipc.cpp:84-160
    for tag in ("<graphics_info>", "<skypos_rac>", "<skypos_dec>", "<dispersion>", "<orb_radius>", "<orb_period>",
                "<orb_phase>", "<power_spectrum>", "<fraction_done>", "<cpu_time>", "<update_time>",
                "<boinc_status>", "<quit_request>", "<max_working_set_size>"):
        assert tag in xml, tag
    # 40-bin screensaver spectrum as two zero-padded hex digits per bin
    import re

    m = re.search(r"<power_spectrum>([0-9a-f]*)</power_spectrum>", xml)
    assert m is not None and len(m.group(1)) == 80


def test_any_padding_has_a_device_plan_and_runs_on_the_golden_model(brp, case, tmp_path):
    # padding 1.3 -> N/2 has a prime factor outside the three-pass FFT's
    # lengths: the HIP backend takes the chirp-z path (no CPU fallback in the
    # product path; GPU parity in tests/test_gpu_bluestein.py), and the CPU
    # golden model (chirp-z double FFT for such lengths) searches it too
    from boinc_app_eah_brp_amd import ops

    cfg = _cfg(case, tmp_path, padding=1.3, use_cpu=True)
    out = BRPSearch(cfg).run(end=3, write_output=False, use_checkpoint=False)
    assert out.templates_run == 3
    N = out.geometry["nsamples"]
    assert brp.fft_plan(N // 2) is None
    assert ops.fft_path(N).kind == "chirp-z"


def test_app_mi355x_flags_parse(app, case, tmp_path):
    """The MI355X option namespace parses without disturbing the BOINC options
    (a flag that did not advance the parser used to hang the app); results
    with --mi355x-spin / --mi355x-ps-fp16 on the CPU backend equal the plain run."""
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    r0 = _run_app(app, _app_args(case, tmp_path / "a"), tmp_path)
    assert r0.returncode == 0, r0.stderr[-2000:]
    r1 = _run_app(app, _app_args(case, tmp_path / "b", ["--mi355x-spin", "--mi355x-batch", "3"]), tmp_path)
    assert r1.returncode == 0, r1.stderr[-2000:]
    assert (tmp_path / "a" / "res.cand").read_text() == (tmp_path / "b" / "res.cand").read_text()
    (tmp_path / "c").mkdir()
    r2 = _run_app(app, _app_args(case, tmp_path / "c", ["--mi355x-ps-fp16", "-h"]), tmp_path)
    assert "--mi355x-spin" in r2.stdout + r2.stderr


def test_app_roctx_ranges_do_not_change_results(app, case, tmp_path):
    """BRP_ROCTX=1 loads the roctx library (dlopen) and brackets the host phases;
    the result file is unchanged."""
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    r1 = _run_app(app, _app_args(case, a), a)
    r2 = _run_app(app, _app_args(case, b), b, BRP_ROCTX="1")
    assert r1.returncode == 0 and r2.returncode == 0, r2.stderr[-2000:]
    assert (a / "res.cand").read_text() == (b / "res.cand").read_text()


def test_fault_spec_parsing(monkeypatch):
    from boinc_app_eah_brp_amd.parallel.dist import fault_param

    monkeypatch.setenv("BRP_FAULT", "hip_oom,collective_timeout:3,kill_after_template:9")
    assert fault_param("collective_timeout") == "3"
    assert fault_param("hip_oom") == ""
    assert fault_param("kill_after_template") == "9"
    assert fault_param("kill_after") is None
    monkeypatch.delenv("BRP_FAULT")
    assert fault_param("hip_oom") is None


def test_app_no_checkpoint_and_progress_every(app, case, tmp_path):
    """--mi355x-no-checkpoint (Debian -DNOCHECKPOINTING) never writes a checkpoint,
    even when interrupted; --mi355x-progress-every (-DCOMMUNICATIONREDUCTION)
    leaves the results unchanged."""
    ref, run, cut = tmp_path / "ref", tmp_path / "run", tmp_path / "cut"
    for d in (ref, run, cut):
        d.mkdir()
    r = _run_app(app, _app_args(case, ref), ref)
    assert r.returncode == 0, r.stderr[-2000:]
    extra = ("--mi355x-no-checkpoint", "--mi355x-progress-every", "5")
    r = _run_app(app, _app_args(case, run, extra), run, BRP_CHECKPOINT_PERIOD="0")
    assert r.returncode == 0, r.stderr[-2000:]
    assert "option ignored" in r.stderr
    assert _result_lines(run / "res.cand") == _result_lines(ref / "res.cand")
    r = _run_app(app, _app_args(case, cut, extra), cut, BRP_CHECKPOINT_PERIOD="0", BRP_FAULT="kill_after_template:5")
    assert r.returncode == 0, r.stderr[-2000:]
    assert not (cut / "cp.cpt").exists() and not (cut / "res.cand").exists()


@pytest.mark.parametrize("batch,workers", [(4, 3), (3, 2), (1, 4)])
def test_session_table_independent_of_batching(brp, case, tmp_path, batch, workers):
    """SearchSession.run deals batches to its workers (shrinking the last ones
    so the pipelines finish together) and applies them in template order: the
    candidate table is byte-identical to one worker with one-template batches
    (demod_binary.c:1180-1443 sequential semantics)."""
    def table(b, w):
        opts = _cfg(case, tmp_path, batch=b).options()
        s = brp.SearchSession()
        s.open(opts, w, [])
        s.prepare()
        t, _ = s.run(0, s.total(), brp.CandidateTable())
        return bytes(t.to_bytes())

    ref = table(1, 1)
    assert table(batch, workers) == ref
