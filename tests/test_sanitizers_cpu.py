"""Host-code sanitizers: the application built with ASan +
UBSan (`python -m boinc_app_eah_brp_amd._build --asan`) runs a full synthetic
search on the CPU backend -- WU/bank/zaplist parsing, whitening, GSL-compatible
RNG, running median, candidate table, checkpoint under fault injection and
resume, result writer, shared-memory telemetry -- with no sanitizer report,
and produces the same result file as the regular build. The ThreadSanitizer
build (`--tsan`) runs the multi-worker search (three CPU workers feeding the
in-order applier, checkpoints, quit and resume) with no race report."""
import os
import subprocess
from pathlib import Path

import pytest

from boinc_app_eah_brp_amd import _build
from boinc_app_eah_brp_amd.utils import synth

INJ = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)


@pytest.fixture(scope="module")
def apps():
    return _build.build(verbose=False)["app"], _build.build_asan(verbose=False)


def _run(app, args, cwd, **env):
    e = dict(os.environ, BRP_NO_RESULT_HEADER="1", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
             UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", **env)
    return subprocess.run([str(app), *args], cwd=cwd, env=e, capture_output=True, text=True, timeout=600)


def test_asan_ubsan_full_search_clean(apps, tmp_path):
    app, asan = apps
    case = synth.synthetic_case(tmp_path, n=1 << 15, n_templates=17, inj=INJ)
    outs = {}
    for name, exe in (("plain", app), ("asan", asan)):
        d = tmp_path / name
        d.mkdir()
        args = ["-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o", str(d / "res.cand"), "-c",
                str(d / "cp.cpt"), "-A", "0.08", "-P", "3.0", "-f", "400.0", "-W", "-B", "100", "--mi355x-cpu",
                "--mi355x-batch", "3"]
        # interrupted run (checkpoint after 7 templates) + resume
        r = _run(exe, args, d, BRP_FAULT="kill_after_template:7", BRP_CHECKPOINT_PERIOD="0")
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        r = _run(exe, args, d)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        outs[name] = (d / "res.cand").read_text()
    assert outs["plain"] == outs["asan"]
    assert "%DONE%" in outs["asan"]


def test_tsan_multi_worker_search_clean(tmp_path):
    """Race detection of the host side: three worker threads (--mi355x-gpus 3
    on the CPU backend) deal batches to the in-order candidate applier, with a
    checkpoint after every batch, a quit after 11 templates and a resume. No
    ThreadSanitizer report, and the result equals the regular build's."""
    app = _build.build(verbose=False)["app"]
    tsan = _build.build_tsan(verbose=False)
    case = synth.synthetic_case(tmp_path, n=1 << 15, n_templates=23, inj=INJ)
    outs = {}
    for name, exe in (("plain", app), ("tsan", tsan)):
        d = tmp_path / name
        d.mkdir()
        args = ["-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o", str(d / "res.cand"), "-c",
                str(d / "cp.cpt"), "-A", "0.08", "-P", "3.0", "-f", "400.0", "-W", "-B", "100", "--mi355x-cpu",
                "--mi355x-gpus", "3", "--mi355x-batch", "2"]
        env = dict(TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1", BRP_CHECKPOINT_PERIOD="0")
        r = _run(exe, args, d, BRP_FAULT="kill_after_template:11", **env)
        assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
        r = _run(exe, args, d, **env)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
        outs[name] = (d / "res.cand").read_text()
    assert outs["plain"] == outs["tsan"]
    assert "%DONE%" in outs["tsan"]
