"""Two-pass FFT plan for the bench geometry (pytest -m gpu): pass A (the
resampling gather and the whole 24576-point column transform,
csrc/hip/fft_two_pass.hip) and pass B (pass 3 on pass A's transposed row
tiles) against the three-pass plan and the CPU golden model. BRP_TWO_PASS is
read at engine setup. (The plan itself is opt-in, BRP_TWO_PASS=1: it runs at
15.2k vs 19.1k templates/s, profiles/two_pass_r4.txt.)"""
import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig

from conftest import BANK, WU, ZAP
from test_gpu_search import _compare_tables

pytestmark = pytest.mark.gpu


def _engine(brp, monkeypatch, tp, geom, series, mu):
    monkeypatch.setenv("BRP_TWO_PASS", tp)
    eng = brp.HipEngine()
    eng.init(0, 1)
    eng.setup(geom, series, mu)
    return eng


def test_two_pass_spectrum_vs_three_pass_and_cpu(brp, gpu, monkeypatch):
    """Shipped WU at -P 3: the two plans' spectra agree to 5e-5 of
    max(P_k, mean P), and the two-pass spectrum is as close to the CPU double
    model as the three-pass one."""
    hdr, series, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=3.0, fA=0.08, window=1000))
    mu = float(np.mean(series.astype(np.float64)))
    e2 = _engine(brp, monkeypatch, "1", geom, series, mu)
    e3 = _engine(brp, monkeypatch, "0", geom, series, mu)
    monkeypatch.setenv("BRP_CPU_MEAN", "double")
    for P, tau, psi in ((1046.6, 0.0547, 4.48), (11000.0, 0.012, 2.5)):
        p2, n2 = e2.power_spectrum(P, tau, psi)
        p3, n3 = e3.power_spectrum(P, tau, psi)
        assert n2 == n3
        xr, _, _ = brp.cpu_resample(series, geom, P, tau, psi)
        pc = brp.cpu_power_spectrum(xr, geom["fft_size"])
        scale = np.maximum(pc[1:], float(np.mean(pc[1:])))
        d23 = np.abs(p2.astype(np.float64) - p3)[1:] / scale
        assert d23.max() < 5e-5, (P, d23.max(), int(np.argmax(d23)))
        e2c = (np.abs(p2.astype(np.float64) - pc)[1:] / scale)[999:].max()
        e3c = (np.abs(p3.astype(np.float64) - pc)[1:] / scale)[999:].max()
        assert e2c < 2e-4 and e2c < 1.5 * e3c + 1e-6, (P, e2c, e3c)


def test_two_pass_search_table_vs_three_pass(brp, gpu, monkeypatch, tmp_path):
    """First 400 templates of the bench configuration: the two-pass table
    equals the three-pass one within float-FFT tolerance (near-ties aside)."""
    tabs = {}
    for tp in ("1", "0"):
        monkeypatch.setenv("BRP_TWO_PASS", tp)
        cfg = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), outputfile=str(tmp_path / f"t{tp}.cand"), batch=1)
        tabs[tp] = BRPSearch(cfg, pipelines=3).run(begin=0, end=400, write_output=False, use_checkpoint=False)
    assert tabs["1"].templates_run == 400
    _compare_tables(tabs["1"].table, tabs["0"].table)
