"""Independent numpy oracle of the per-template pipeline (float64 FFT).

Written directly from the reference semantics (not from the C++ golden model)
so the two CPU implementations cross-check each other:
  resampling      demod_binary_resamp_cpu.c:80-136 (+ LUT sine, erp_utilities.cpp:176-209)
  power spectrum  demod_binary_fft_fftw.c:88-113
  harmonic sums   hs_common.c:33-171
Vectorised, so it is usable up to ~2^20-sample series in tests.
"""
from __future__ import annotations

import math

import numpy as np

from .. import native


def lut_tables():
    s, c = native().lut_tables()
    return np.asarray(s, np.float32), np.asarray(c, np.float32)


def lut_sin(x: np.ndarray) -> np.ndarray:
    """Vectorised float32 LUT sine with the reference's operation order."""
    s_lut, c_lut = lut_tables()
    x = np.asarray(x, np.float32)
    two_pi = np.float32(6.283185)
    inv = np.float32(1.0) / two_pi
    xt = np.float32(inv * x)
    xt = np.float32(xt - np.trunc(xt))
    xt = np.where(xt < 0, np.float32(xt + np.float32(1.0)), xt).astype(np.float32)
    i0 = (xt * np.float32(64.0) + np.float32(0.5)).astype(np.int32)
    d = np.float32(two_pi * np.float32(xt - np.float32(1.0 / 64.0) * i0.astype(np.float32)))
    d2 = np.float32(d * np.float32(np.float32(0.5) * d))
    ts, tc = s_lut[i0], c_lut[i0]
    return np.float32(np.float32(ts + np.float32(d * tc)) - np.float32(d2 * ts))


def resample(series: np.ndarray, geom: dict, P: float, tau: float, psi0: float):
    """Returns (resampled padded series, n_steps, mean)."""
    nu = int(geom["n_unpadded"])
    n = int(geom["nsamples"])
    dt = np.float32(geom["dt"])
    step_inv = np.float32(geom["step_inv"])
    P, tau, psi0 = np.float32(P), np.float32(tau), np.float32(psi0)
    omega = np.float32(2.0 * math.pi / float(P))
    S0 = np.float32(np.float32(tau * np.float32(math.sin(float(psi0)))) * step_inv)
    i = np.arange(nu, dtype=np.float32)
    t = np.float32(i * dt)
    s = lut_sin(np.float32(np.float32(omega * t) + psi0))
    del_t = np.float32(np.float32(np.float32(tau * s) * step_inv) - S0)
    n_steps = nu - 1
    while np.float32(np.float32(n_steps) - del_t[n_steps]) >= np.float32(nu - 1):
        n_steps -= 1
    idx = (np.float32(i[:n_steps] - del_t[:n_steps]).astype(np.float64) + 0.5).astype(np.int64)
    out = np.empty(n, np.float32)
    out[:n_steps] = series[np.clip(idx, 0, nu - 1)]
    # sequential float accumulation, divided by the float sample count
    # (demod_binary_resamp_cpu.c:112-125); cumsum is sequential, sum is pairwise
    mean = np.float32(np.cumsum(out[:n_steps], dtype=np.float32)[-1] / np.float32(n_steps))
    out[n_steps:] = mean
    return out, n_steps, mean


def power_spectrum(x: np.ndarray, fft_size: int) -> np.ndarray:
    X = np.fft.rfft(x.astype(np.float64))[:fft_size]
    ps = (np.abs(X) ** 2 / x.size).astype(np.float32)
    ps[0] = 0.0
    return ps


def harmonic_sums(ps: np.ndarray, geom: dict, thr=None) -> np.ndarray:
    """sumspec[h][j] for h=0..4, j < fundamental_idx_hi (reference float order).

    Without `thr`: the max of S_h(i) over the cell's i. With `thr`: the
    reference's exact array contents (hs_common.c:78-165) -- a cell is
    rewritten only on its first visit or when the running max exceeds thr[h],
    so cells whose max stays <= thr[h] keep the first visited S_h(i)."""
    w2, fhi, hhi = int(geom["window_2"]), int(geom["fundamental_idx_hi"]), int(geom["harmonic_idx_hi"])
    i = np.arange(w2, hhi, dtype=np.int64)
    P = ps.astype(np.float32)

    def g(k):
        return P[(k * i + 8) >> 4]

    s = g(16)
    s = np.float32(s + g(8))
    S1 = s
    s = np.float32(s + np.float32(g(12) + g(4)))
    S2 = s
    s = np.float32(s + np.float32(np.float32(np.float32(g(14) + g(10)) + g(6)) + g(2)))
    S3 = s
    acc = g(15)
    for k in (13, 11, 9, 7, 5, 3, 1):
        acc = np.float32(acc + g(k))
    s = np.float32(s + acc)
    S4 = s
    out = np.zeros((5, fhi), np.float32)
    out[0] = P[:fhi]
    for h, S in ((1, S1), (2, S2), (3, S3), (4, S4)):
        j = (i + (1 << (h - 1))) >> h
        m = j < fhi
        np.maximum.at(out[h], j[m], S[m])
        if thr is not None:
            jj, first = np.unique(j[m], return_index=True)
            low = out[h][jj] <= np.float32(thr[h])
            out[h][jj[low]] = np.maximum(S[m][first[low]], np.float32(0.0))
    return out


def candidates(sumspec: np.ndarray, geom: dict, thr) -> list:
    """Per level the (bins, powers) above thr in [window_2, fundamental_idx_hi)."""
    w2 = int(geom["window_2"])
    res = []
    for h in range(5):
        v = sumspec[h]
        b = np.nonzero(v[w2:] > np.float32(thr[h]))[0] + w2
        res.append((b.astype(np.uint32), v[b]))
    return res
