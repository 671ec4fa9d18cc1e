"""Every padding the reference accepts on the GPU (pytest -m gpu).

The reference takes any -P in [1, 10] and FFTs nsamples = (int)(P*N_u + 0.5)
samples (demod_binary.c:226-244, 782; cuFFT/FFTW plan any length). Lengths the
three-pass FFT does not factor (odd N, or N/2 with a prime factor above 5) run
as a chirp-z transform on the device (csrc/hip/bluestein.hip); these tests pin
it against the double-precision CPU model (whose FFT is itself a chirp-z
convolution for such lengths, checked against numpy in
tests/test_numerics.py)."""
import os
import subprocess

import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth

pytestmark = pytest.mark.gpu

INJ = synth.Injection(f0=97.0, P_orb=700.0, tau=0.02, psi0=0.3, amplitude=2.0)


def _geom(brp, tmp_path, n, padding, window=100, f0=150.0):
    x = synth.make_series(n, 65.476, INJ)
    wu = synth.write_wu(tmp_path / "a.bin4", x)
    hdr, series, _ = brp.read_work_unit(str(wu))
    geom = brp.derive_geometry(hdr, dict(f0=f0, padding=padding, fA=0.08, window=window))
    return hdr, series, geom


@pytest.mark.parametrize("n,padding", [(1 << 16, 1.1), (1 << 16, 1.7), (1 << 17, 2.3), (1 << 18, 9.9),
                                       (1 << 16, 3.01)])
def test_power_spectrum_any_padding(brp, gpu, tmp_path, n, padding):
    """Non-smooth and odd N: the device spectrum (chirp-z) matches the CPU
    double-precision spectrum, with n_steps and the mean padding exact."""
    _, series, geom = _geom(brp, tmp_path, n, padding)
    N = geom["nsamples"]
    assert brp.fft_plan(N // 2) is None or N % 2, (N, "expected a length outside the three-pass set")
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
        assert err.max() < 2e-4, (N, padding, err.max(), int(np.argmax(err)) + 1)


@pytest.mark.parametrize("padding", [1.1, 1.7])
def test_whitening_any_padding(brp, gpu, tmp_path, padding):
    """Device whitening (forward chirp-z, running median, zapping, inverse
    chirp-z; odd N via the Hermitian extension) matches the CPU whitening."""
    case = synth.synthetic_case(tmp_path, n=1 << 16, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    opt = dict(f0=200.0, padding=padding, fA=0.08, window=200, white=True)
    geom = brp.derive_geometry(hdr, opt)
    zaps = brp.read_zaplist(case["zap"])
    w_cpu = brp.cpu_whiten(series, geom, opt, zaps)
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, series, 0.0)
    w_gpu = eng.whiten(opt, zaps, series)
    rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
    assert rms > 0
    assert np.max(np.abs(w_gpu - w_cpu)) / rms < 1e-4, (padding, geom["nsamples"])


@pytest.mark.parametrize("padding", [1.7, 2.3])
def test_search_any_padding_matches_cpu(brp, gpu, tmp_path, padding):
    """Whole searches at paddings outside the three-pass set: GPU candidate
    table equals the CPU golden model's (same bins, powers within float-FFT
    tolerance)."""
    from test_gpu_search import _compare_tables

    inj = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "c", n=1 << 16, n_templates=12, inj=inj)
    cfg = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0, padding=padding,
               fA=0.08, window=100, white=True, batch=2)
    g = BRPSearch(SearchConfig(outputfile=str(tmp_path / "g.cand"), **cfg)).run(use_checkpoint=False)
    c = BRPSearch(SearchConfig(outputfile=str(tmp_path / "c.cand"), use_cpu=True, **cfg), gpus=8).run(
        use_checkpoint=False)
    assert g.templates_run == c.templates_run == 13
    _compare_tables(g.table, c.table)


def test_app_any_padding_runs_on_gpu(brp, gpu, tmp_path):
    """The BOINC application at -P 1.7 stays on the HIP backend (no CPU
    fallback) and writes a complete result file."""
    inj = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "c", n=1 << 16, n_templates=6, inj=inj)
    args = [str(app_binary()), "-i", case["wu"], "-t", case["bank"], "-l", case["zap"], "-o",
            str(tmp_path / "r.cand"), "-c", str(tmp_path / "cp.cpt"), "-A", "0.08", "-P", "1.7", "-f", "400.0",
            "-W", "-B", "100"]
    r = subprocess.run(args, cwd=tmp_path, env=dict(os.environ, BRP_NO_RESULT_HEADER="1"), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "chirp-z transform" in r.stderr and "CPU backend" not in r.stderr
    lines, done = brp.read_results(str(tmp_path / "r.cand"))
    assert done and lines


@pytest.mark.parametrize("padding", [2.7, 2.9])
def test_power_spectrum_bench_size(brp, gpu, padding, monkeypatch):
    """Production size: the shipped 2^22-sample WU at -P 2.7 (N = 11 324 621,
    odd: a chirp-z DFT of length N over L >= 2N - 1) and -P 2.9 (N = 12 163 482,
    N/2 = 3 * 2 027 247: the packed even path). The device spectrum of two
    templates against the CPU double-precision spectrum, same bound as the
    small lengths (the fp32 convolution error grows with L).

    The series is raw (~5e4 per sample), so the CPU model pads with the
    accurate mean (BRP_CPU_MEAN=double), as the device and the reference's
    CUDA build do: the reference CPU build's serial float sum is 1.8 % off
    here (48 688 vs 47 827), which alone moves bin 147 by 58 %."""
    from conftest import WU

    monkeypatch.setenv("BRP_CPU_MEAN", "double")

    hdr, series, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=padding, fA=0.08, window=1000))
    N = geom["nsamples"]
    assert brp.fft_plan(N // 2) is None or N % 2, N
    eng = brp.HipEngine()
    eng.init(0, 1)
    eng.setup(geom, series, float(np.mean(series)))
    for P, tau, psi in ((1046.6, 0.0547, 4.48), (2000.0, 0.3, 1.0)):
        ps_g, ns_g = eng.power_spectrum(P, tau, psi)
        xr, ns_c, _ = brp.cpu_resample(series, geom, P, tau, psi)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        assert ns_g == ns_c
        scale = float(np.mean(ps_c[1:]))
        err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
        assert err.max() < 2e-4, (N, padding, err.max(), int(np.argmax(err)) + 1)


@pytest.mark.parametrize("fA,end,golden", [(0.08, 50, "bench_wu_cpu_table_first50_P2.7.bin"),
                                            (0.9999, 24, "bench_wu_cpu_table_first24_A0.9999_P2.7.bin")])
def test_bench_wu_p27_prefix_vs_cpu_golden(brp, gpu, fA, end, golden):
    """The shipped WU at -P 2.7 -W (chirp-z path at bench size, odd N: two
    templates per transform), first templates against the CPU golden model
    (tools/make_golden.py --end 50 --padding 2.7; --end 24 --fA 0.9999 for a
    table with candidates on every level)."""
    from conftest import BANK, ROOT, WU, ZAP
    from test_gpu_search import _compare_tables

    cfg = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), batch=1)
    cfg.padding = 2.7
    cfg.fA = fA
    g = BRPSearch(cfg, pipelines=3).run(begin=0, end=end, write_output=False, use_checkpoint=False)
    assert g.templates_run == end and g.geometry["nsamples"] == 11324621
    gold = brp.CandidateTable()
    gold.from_bytes(np.frombuffer((ROOT / "data" / "golden" / golden).read_bytes(), dtype=np.uint8).copy())
    assert sum(1 for e in gold.entries() if e[5] > 0) >= (1 if fA < 0.5 else 40)
    _compare_tables(g.table, gold)


def test_odd_length_template_pairs_match_single(brp, gpu, tmp_path, monkeypatch):
    """Odd N runs two templates per chirp-z transform (x_a + i x_b, separated
    by conjugate symmetry; P1_CHIRP1_PAIR): the candidate table matches the
    one-template-per-transform path (BRP_BS_PAIR=0) and the CPU golden model,
    with an odd number of templates per launch group (13 templates, groups of 2
    and 3)."""
    from test_gpu_search import _compare_tables

    inj = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)
    case = synth.synthetic_case(tmp_path / "c", n=1 << 16, n_templates=12, inj=inj)
    for batch in (2, 3):
        cfg = dict(inputfile=case["wu"], templatebank=case["bank"], zaplistfile=case["zap"], f0=400.0,
                   padding=2.3, fA=0.08, window=100, white=True, batch=batch)
        pair = BRPSearch(SearchConfig(**cfg)).run(write_output=False, use_checkpoint=False)
        monkeypatch.setenv("BRP_BS_PAIR", "0")
        single = BRPSearch(SearchConfig(**cfg)).run(write_output=False, use_checkpoint=False)
        monkeypatch.delenv("BRP_BS_PAIR")
        assert pair.geometry["nsamples"] % 2 == 1
        _compare_tables(pair.table, single.table, rtol=1e-5)
        c = BRPSearch(SearchConfig(use_cpu=True, **cfg), gpus=8).run(write_output=False, use_checkpoint=False)
        _compare_tables(pair.table, c.table)


# (samples, padding) whose chirp-z plans put every length of the
# register-staged passes in place at least once: pass1g_kernel for L1 (48 ...
# 512, forward P1_CHIRP* and the transposed inverse's P1_REV_CHIRP), pass 2
# for L2 forward and reversed (pass2r_kernel 32 / 64 / 128 / 256,
# pass2g_kernel 48 ... 320; 384 ... 512 need more than 2^21 samples),
# pass3_mid_kernel for every L3. Plans with L1 or L2 = 16 (e.g. 1.13 and 1.53
# at 2^16) run the natural-order convolution. Found with derive_geometry +
# brp.bluestein_plan (the cost model of make_bluestein_plan); asserted below.
_REG_CASES = [
    (1 << 16, 1.03, (48, 16, 96)), (1 << 16, 1.13, (16, 16, 320)), (1 << 16, 1.53, (112, 16, 64)),
    (1 << 16, 1.78, (48, 16, 160)), (1 << 16, 1.33, (48, 48, 96)), (1 << 16, 1.7, (112, 16, 128)),
    (1 << 16, 1.76, (48, 32, 192)), (1 << 16, 3.39, (64, 32, 256)), (1 << 16, 4.51, (80, 32, 256)),
    (1 << 16, 5.01, (144, 48, 96)), (1 << 16, 6.01, (112, 112, 64)), (1 << 16, 7.51, (64, 64, 256)),
    (1 << 16, 8.01, (96, 48, 256)), (1 << 17, 6.13, (80, 80, 256)), (1 << 17, 7.51, (128, 64, 256)),
    (1 << 17, 8.76, (96, 96, 256)), (1 << 18, 6.13, (160, 80, 256)), (1 << 18, 7.88, (128, 128, 256)),
    (1 << 18, 9.02, (240, 80, 256)), (1 << 19, 5.01, (144, 144, 256)), (1 << 19, 5.08, (192, 112, 256)),
    (1 << 19, 6.01, (224, 112, 256)), (1 << 19, 6.15, (160, 160, 256)), (1 << 19, 7.9, (256, 128, 256)),
    (1 << 19, 8.76, (192, 192, 256)), (1 << 20, 5.04, (288, 144, 256)), (1 << 20, 6.04, (224, 224, 256)),
    (1 << 20, 6.13, (320, 160, 256)), (1 << 20, 7.88, (256, 256, 256)), (1 << 21, 7.01, (240, 240, 256)),
    (1 << 21, 5.02, (288, 288, 256)), (1 << 21, 5.07, (384, 224, 256)), (1 << 21, 6.02, (448, 224, 256)),
    (1 << 21, 6.14, (320, 320, 256)), (1 << 21, 7.89, (512, 256, 256)),
]


@pytest.mark.parametrize("n,padding,l12", _REG_CASES)
def test_register_staged_pass_lengths(brp, gpu, tmp_path, monkeypatch, n, padding, l12):
    """Every L1 / L2 of the register-staged chirp-z passes: the device
    spectrum of one template against the CPU double-precision spectrum (the
    CPU model pads with the accurate mean, as the device does: at 2^21 samples
    the reference CPU build's serial float mean moves the lowest bins)."""
    monkeypatch.setenv("BRP_CPU_MEAN", "double")
    _, series, geom = _geom(brp, tmp_path, n, padding)
    N = geom["nsamples"]
    plan = brp.bluestein_plan(N if N % 2 else N // 2)
    assert plan is not None and tuple(plan[1:4]) == l12, (N, plan)
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, series, float(np.mean(series)))
    ps_g, ns_g = eng.power_spectrum(900.0, 0.05, 1.3)
    xr, ns_c, _ = brp.cpu_resample(series, geom, 900.0, 0.05, 1.3)
    ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
    assert ns_g == ns_c
    scale = float(np.mean(ps_c[1:]))
    err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
    assert err.max() < 2e-4, (N, padding, l12, err.max(), int(np.argmax(err)) + 1)
