"""Paddings whose FFT length is 7-smooth (pytest -m gpu): N/2 = 7 * 2^k, e.g.
-P 3.5 (N = 7 * 2^21 at the benchmark's 2^22 samples) or -P 6.125, factor
over the radix-7 plan lengths (112 = 7 * 16, 224 = 2 * 7 * 16, 448) and take
the three-pass path (pass1g_kernel's resampling gather, pass2g_kernel)
instead of a chirp-z transform over a length >= 2N - 1. cuFFT plans such
lengths directly (cuda/app/demod_binary_cuda.cu:863); the reference accepts
any -P in [1, 10] (demod_binary.c:226-244, 782). Device spectra against the
CPU double-precision spectrum, whitening against the CPU whitening, and the
shipped WU at -P 3.5 against the CPU golden table
(tools/make_golden.py --end 50 --padding 3.5)."""
import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.utils import synth

pytestmark = pytest.mark.gpu

INJ = synth.Injection(f0=97.0, P_orb=700.0, tau=0.02, psi0=0.3, amplitude=2.0)

# (samples, padding, plan (L1, L2, L3)): every radix-7 length as L1 and as L2
_CASES = [(1 << 16, 3.5, (112, 16, 64)), (1 << 18, 6.125, (112, 112, 64)), (1 << 21, 6.125, (224, 112, 256))]


def _spectra_match(brp, eng, series, geom, templates):
    for P, tau, psi in templates:
        ps_g, ns_g = eng.power_spectrum(P, tau, psi)
        xr, ns_c, _ = brp.cpu_resample(series, geom, P, tau, psi)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        assert ns_g == ns_c
        scale = float(np.mean(ps_c[1:]))
        err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
        assert err.max() < 2e-4, (geom["nsamples"], err.max(), int(np.argmax(err)) + 1)


@pytest.mark.parametrize("n,padding,plan", _CASES)
def test_radix7_power_spectrum(brp, gpu, tmp_path, monkeypatch, n, padding, plan):
    monkeypatch.setenv("BRP_CPU_MEAN", "double")
    x = synth.make_series(n, 65.476, INJ)
    wu = synth.write_wu(tmp_path / "a.bin4", x)
    hdr, series, _ = brp.read_work_unit(str(wu))
    geom = brp.derive_geometry(hdr, dict(f0=150.0, padding=padding, fA=0.08, window=100))
    N = geom["nsamples"]
    assert tuple(brp.fft_plan(N // 2))[:3] == plan, (N, brp.fft_plan(N // 2))
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, series, float(np.mean(series)))
    _spectra_match(brp, eng, series, geom, ((700.0, 0.02, 0.3), (1500.0, 0.3, 4.0)))


@pytest.mark.parametrize("n,padding", [(1 << 16, 3.5), (1 << 18, 6.125)])
def test_radix7_whitening(brp, gpu, tmp_path, n, padding):
    """Whitening's forward real FFT (LDS-staged pass 1 over Radices<112 / 224>)
    and inverse transform at 7-smooth N match the CPU whitening."""
    case = synth.synthetic_case(tmp_path, n=n, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    opt = dict(f0=200.0, padding=padding, fA=0.08, window=200, white=True)
    geom = brp.derive_geometry(hdr, opt)
    assert brp.fft_plan(geom["nsamples"] // 2) is not None
    zaps = brp.read_zaplist(case["zap"])
    w_cpu = brp.cpu_whiten(series, geom, opt, zaps)
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, series, 0.0)
    w_gpu = eng.whiten(opt, zaps, series)
    rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
    assert rms > 0
    assert np.max(np.abs(w_gpu - w_cpu)) / rms < 1e-4, (padding, geom["nsamples"])


def test_radix7_bench_size_spectrum(brp, gpu, monkeypatch):
    """The shipped 2^22-sample WU at -P 3.5: N = 14 680 064, plan
    224 x 128 x 256 (pass1g_kernel<224> resampling gather); spectra of two
    templates against the CPU double-precision spectrum (raw series: the CPU
    model pads with the accurate mean, like the device)."""
    from conftest import WU

    monkeypatch.setenv("BRP_CPU_MEAN", "double")
    hdr, series, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=3.5, fA=0.08, window=1000))
    assert geom["nsamples"] == 14680064
    assert tuple(brp.fft_plan(geom["nsamples"] // 2))[:3] == (224, 128, 256)
    eng = brp.HipEngine()
    eng.init(0, 1)
    eng.setup(geom, series, float(np.mean(series)))
    _spectra_match(brp, eng, series, geom, ((1046.6, 0.0547, 4.48), (2000.0, 0.3, 1.0)))


def test_bench_wu_p35_prefix_vs_cpu_golden(brp, gpu):
    """-P 3.5 -W on the shipped WU, first 50 templates, three pipelines:
    the candidate table equals the CPU golden model's."""
    from conftest import BANK, ROOT, WU, ZAP
    from test_gpu_search import _compare_tables

    cfg = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), batch=1)
    cfg.padding = 3.5
    g = BRPSearch(cfg, pipelines=3).run(begin=0, end=50, write_output=False, use_checkpoint=False)
    assert g.templates_run == 50 and g.geometry["nsamples"] == 14680064
    gold = brp.CandidateTable()
    gold.from_bytes(np.frombuffer((ROOT / "data" / "golden" / "bench_wu_cpu_table_first50_P3.5.bin").read_bytes(),
                                  dtype=np.uint8).copy())
    assert sum(1 for e in gold.entries() if e[5] > 0) >= 1
    _compare_tables(g.table, gold)
