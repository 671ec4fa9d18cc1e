"""Numerical building blocks: chi^2 thresholds (GSL cdf replacements), GSL
taus2 / ziggurat, running median, LUT sine, CPU FFT."""
import math

import numpy as np
import pytest
from scipy import stats


def test_chisq_Q_matches_scipy(brp):
    for dof in (2, 4, 8, 16, 32):
        for x in (0.5, 3.0, 10.0, 40.0, 90.0, 200.0):
            want = stats.chi2.sf(x, dof)
            got = brp.chisq_Q_even(x, dof // 2)  # k = dof / 2
            assert math.isclose(got, want, rel_tol=1e-10, abs_tol=1e-300), (x, dof)


def test_chisq_Qinv_inverts(brp):
    for dof in (2, 4, 8, 16, 32):
        for q in (1e-3, 1e-7, 8.48e-7, 1e-12, 3e-14):
            x = brp.chisq_Qinv_even(q, dof // 2)
            assert math.isclose(stats.chi2.isf(q, dof), x, rel_tol=1e-9)


def test_benchmark_thresholds(brp):
    # -A 0.08 on the benchmark geometry (fft_size 6291457):
    # 0.5 * Qinv(prob, 2*2^h) for h = 0..4
    prob = brp.single_bin_probability(0.08, 6291457)
    thr = brp.power_thresholds(prob)
    want = [18.139, 21.241, 26.269, 34.648, 48.958]
    np.testing.assert_allclose(thr, want, atol=2e-3)


def test_candidate_significance(brp):
    # -log10 of the false-alarm probability of the summed power
    for nh in (1, 2, 4, 8, 16):
        p = 30.0
        want = -math.log10(stats.chi2.sf(2 * p, 2 * nh))
        assert math.isclose(brp.candidate_significance(p, nh), want, rel_tol=1e-6)
    # below DBL_MIN the reference clamps to 320
    assert brp.candidate_significance(1000.0, 1) == 320.0


def test_taus2_gsl_sequence(brp):
    # GSL's own regression value: 10000th output of taus2 with the default seed
    r = brp.Taus2(0)
    v = 0
    for _ in range(10000):
        v = r.get()
    assert v == 2733957125
    r.set(1)
    a = [r.get() for _ in range(5)]
    r.set(1)
    assert a == [r.get() for _ in range(5)]


def test_ziggurat_moments(brp):
    r = brp.Taus2(12345)
    x = np.array([brp.gaussian_ziggurat(r, 1.0) for _ in range(200000)])
    assert abs(x.mean()) < 0.01
    assert abs(x.std() - 1.0) < 0.01
    assert abs(stats.kurtosis(x)) < 0.05
    # tails are produced (the ziggurat's base strip)
    assert (np.abs(x) > 3.5).sum() > 10
    r2 = brp.Taus2(12345)
    assert brp.gaussian_ziggurat(r2, 2.0) == pytest.approx(2.0 * x[0])


@pytest.mark.parametrize("w", [1, 2, 5, 16, 101, 1000])
def test_running_median(brp, w):
    rng = np.random.default_rng(w)
    x = rng.exponential(1.0, 4000).astype(np.float32)
    got = brp.running_median(x, w)
    win = np.lib.stride_tricks.sliding_window_view(x, w)
    srt = np.sort(win, axis=1)
    if w % 2:
        want = srt[:, w // 2]
    else:
        # even window: float average of the two middle elements
        want = ((srt[:, w // 2 - 1].astype(np.float32) + srt[:, w // 2]) / np.float32(2.0)).astype(np.float32)
    np.testing.assert_array_equal(got, want)


def test_lut_sin(brp):
    from boinc_app_eah_brp_amd.models import reference

    x = np.linspace(-50, 50, 20001).astype(np.float32)
    got = np.array([brp.lut_sin(float(v)) for v in x[::50]], np.float32)
    np.testing.assert_allclose(got, np.sin(x[::50].astype(np.float64)), atol=2e-5)
    # vectorised oracle reproduces the scalar native implementation bit for bit
    np.testing.assert_array_equal(reference.lut_sin(x[::50]), got)


@pytest.mark.parametrize("n", [16, 96, 1000, 3 * 2 ** 12, 2 * 3 * 5 * 7 * 11,
                               1009, 2 * 1009, 72090, 111411, 3 * 65537])
def test_cpu_rfft(brp, n):
    """Double-precision golden FFT against numpy, including the lengths any
    padding -P produces (prime factors above 64 run as a chirp-z
    convolution, csrc/core/cpu_fft.cpp)."""
    rng = np.random.default_rng(n)
    x = rng.normal(size=n)
    X = brp.rfft(x)
    np.testing.assert_allclose(X, np.fft.rfft(x), rtol=0, atol=1e-9 * n)
    y = brp.irfft(X, n)
    # unnormalised c2r (FFTW semantics): n * x
    np.testing.assert_allclose(y, x * n, atol=1e-8 * n)


@pytest.mark.parametrize("padding", [1.0, 3.0])
def test_n_steps_search_equals_reference_scan(brp, padding):
    """The bracketed n_steps search uploaded by the HIP engine equals the
    reference's descending scan (demod_binary_resamp_cpu.c:94-99) for every
    template of the benchmark bank and for extreme synthetic orbits."""
    from conftest import BANK, WU

    hdr, _, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=padding, fA=0.08, window=1000))
    P, tau, psi = brp.read_template_bank(str(BANK))
    P, tau, psi = (np.asarray(v, dtype=np.float32) for v in (P, tau, psi))
    fast = brp.n_steps(geom, P, tau, psi)
    ref = brp.n_steps(geom, P, tau, psi, scan=True)
    assert np.array_equal(fast, ref)
    rng = np.random.default_rng(5)
    n = 4000
    Ps = rng.uniform(300.0, 5000.0, n).astype(np.float32)
    taus = rng.uniform(0.0, 2.0, n).astype(np.float32)
    psis = rng.uniform(0.0, 2 * np.pi, n).astype(np.float32)
    assert np.array_equal(brp.n_steps(geom, Ps, taus, psis), brp.n_steps(geom, Ps, taus, psis, scan=True))
