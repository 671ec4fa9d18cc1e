"""BOINC integration of the application binary in standalone mode
(SURVEY.md 7.1 shim list): init_data.xml user/host details in the result
header, fraction_done progress file, graphics shared memory, multi-pass
wrapper, debug output."""
import os
import subprocess
from pathlib import Path

import pytest

from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth


@pytest.fixture(scope="module")
def app(brp):
    p = app_binary()
    if not p.exists():
        from boinc_app_eah_brp_amd import _build

        _build.build()
    return p


@pytest.fixture(scope="module")
def small(tmp_path_factory):
    d = tmp_path_factory.mktemp("boinc")
    return synth.synthetic_case(d, n=1 << 14, n_templates=6,
                                inj=synth.Injection(f0=120.0, P_orb=900.0, tau=0.01, psi0=1.0, amplitude=3.0))


def _args(c, out, cp, extra=()):
    return ["-i", c["wu"], "-t", c["bank"], "-l", c["zap"], "-o", str(out), "-c", str(cp), "-A", "0.08", "-P", "1.0",
            "-f", "400.0", "-W", "-B", "50", "--mi355x-cpu", *extra]


def _run(app, args, cwd, **env):
    return subprocess.run([str(app), *args], cwd=cwd, env=dict(os.environ, **env), capture_output=True, text=True,
                          timeout=300)


def test_init_data_header_and_progress(app, small, tmp_path):
    (tmp_path / "init_data.xml").write_text(
        "<app_init_data>\n<userid>4242</userid>\n<user_name>Jocelyn</user_name>\n<hostid>77</hostid>\n"
        "<host_cpid>abcdef0123</host_cpid>\n<checkpoint_period>0</checkpoint_period>\n</app_init_data>\n")
    prog = tmp_path / "progress.txt"
    r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt"), tmp_path, BRP_PROGRESS_FILE=str(prog))
    assert r.returncode == 0, r.stderr[-2000:]
    text = (tmp_path / "r.cand").read_text()
    assert "% User: 4242 (Jocelyn)" in text and "% Host: 77 (abcdef0123)" in text
    assert "% Exec: einsteinbinary_mi355x" in text and text.rstrip().endswith("%DONE%")
    # fraction_done = (counter + 1) / total exceeds 1 at the end (reference quirk)
    assert float(prog.read_text()) >= 1.0


def test_graphics_shared_memory_file(app, small, tmp_path):
    r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt"), tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    shm = tmp_path / "boinc_EinsteinRadio_0"
    assert shm.exists()
    xml = shm.read_bytes().split(b"\0")[0].decode()
    assert "<graphics_info>" in xml and "<fraction_done>" in xml and "<dispersion>" in xml


def test_graphics_shared_memory_named_after_slot(app, small, tmp_path):
    """libboinc names the graphics segment boinc_<app>_<slot> after
    init_data.xml's slot (erp_boinc_ipc.cpp:188 via boinc_graphics_make_shmem)."""
    (tmp_path / "init_data.xml").write_text("<app_init_data>\n<slot>3</slot>\n</app_init_data>\n")
    r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt"), tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "boinc_EinsteinRadio_3").exists()
    assert not (tmp_path / "boinc_EinsteinRadio_0").exists()


def test_multi_pass_wrapper(app, small, tmp_path):
    # two -i/-o pairs processed as sequential passes; the checkpoint is removed after each
    args = ["-i", small["wu"], "-o", str(tmp_path / "a.cand"), "-i", small["wu"], "-o", str(tmp_path / "b.cand"),
            "-t", small["bank"], "-l", small["zap"], "-c", str(tmp_path / "c.cpt"), "-A", "0.08", "-P", "1.0",
            "-f", "400.0", "-W", "-B", "50", "--mi355x-cpu"]
    r = _run(app, args, tmp_path, BRP_NO_RESULT_HEADER="1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "a.cand").read_text() == (tmp_path / "b.cand").read_text()
    assert not (tmp_path / "c.cpt").exists()


def test_debug_flag_prints_thresholds(app, small, tmp_path):
    r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt", ["-z"]), tmp_path)
    assert r.returncode == 0
    out = r.stdout + r.stderr
    for name in ("thr1", "thr2", "thr4", "thr8", "thr16"):
        assert name in out


def test_help_and_bad_values(app, small, tmp_path):
    # like the reference wrapper, -h reaches MAIN only within a pass: MAIN
    # prints its usage and returns RADPUL_EMISC
    r = _run(app, _args(small, tmp_path / "h.cand", tmp_path / "h.cpt", ["-h"]), tmp_path)
    assert "--input_file" in r.stdout and r.returncode != 0
    assert not (tmp_path / "h.cand").exists()
    for bad in (["-P", "0.5"], ["-P", "11"], ["-A", "2"], ["-f", "-1"], ["-B", "-3"]):
        r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt", bad), tmp_path)
        assert r.returncode != 0, bad


def test_app_info_template_is_valid():
    """data/boinc/app_info.xml.in (anonymous-platform descriptor) is well formed
    and names an AMD GPU coprocessor and options the application accepts."""
    import xml.etree.ElementTree as ET
    from pathlib import Path

    root = ET.parse(Path(__file__).resolve().parent.parent / "data" / "boinc" / "app_info.xml.in").getroot()
    av = root.find("app_version")
    assert av.find("coproc/type").text == "ATI"
    assert av.find("file_ref/file_name").text == root.find("file_info/name").text
    assert av.find("cmdline").text.split()[0] == "--mi355x-pipelines"


def test_debug_buffer_dumps(app, small, tmp_path):
    """-z with --mi355x-dump-dir writes the searched (whitened) series and
    template 0's resampled series and power spectrum, one "%e" value per line
    (reference dumpFloatBufferToTextFile, erp_utilities.cpp:216-233)."""
    import numpy as np

    dump = tmp_path / "dump"
    dump.mkdir()
    r = _run(app, _args(small, tmp_path / "r.cand", tmp_path / "c.cpt", ["-z", "--mi355x-dump-dir", str(dump)]),
             tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    series = np.loadtxt(dump / "dump_series.txt")
    x = np.loadtxt(dump / "dump_resampled_t0.txt")
    ps = np.loadtxt(dump / "dump_power_t0.txt")
    assert len(x) == 2 * (len(ps) - 1) or len(x) == 2 * len(ps) - 1
    assert len(series) <= len(x)
    # the dumped spectrum is the normalised power of the dumped resampled series
    ref = np.abs(np.fft.rfft(x.astype(np.float64))) ** 2 / len(x)
    ref[0] = 0.0
    scale = ref[1:].mean()
    assert np.max(np.abs(ps - ref[:len(ps)]) / np.maximum(ref[:len(ps)], scale)) < 1e-3
    first = (dump / "dump_power_t0.txt").read_text().splitlines()[1]
    assert "e" in first  # "%e" format
