"""C++ golden model (csrc/core/cpu_backend.cpp) against the independent numpy
oracle (models/reference.py), stage by stage, plus the candidate table's
sequential semantics (demod_binary.c:1310-1397) against a literal Python
transcription of that loop."""
import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import reference


def _geom(brp, n=1 << 15, padding=3.0, f0=400.0, window=100, tsample=65.476, fA=0.08):
    hdr = dict(tsample=tsample, nsamples=n, tobs=n * tsample * 1e-6, scale=1.0)
    return brp.derive_geometry(hdr, dict(f0=f0, padding=padding, window=window, fA=fA))


def test_geometry_benchmark(brp):
    # the benchmark WU with -P 3.0 -f 400.0 -A 0.08 (bench geometry)
    from conftest import WU

    hdr, _, _ = brp.read_work_unit(str(WU))
    g = brp.derive_geometry(hdr, dict(f0=400.0, padding=3.0, window=1000, fA=0.08))
    assert g["n_unpadded"] == 1 << 22
    assert g["nsamples"] == 3 << 22
    assert g["fft_size"] == 6291457
    assert g["window_2"] == 500
    assert g["fundamental_idx_hi"] == 329552
    assert g["harmonic_idx_hi"] == 5272839


@pytest.mark.parametrize("tpl", [(1000.0, 0.0, 0.0), (700.5, 0.3, 1.0), (2200.0, 0.12, 5.9), (660.0, 0.335, 3.14)])
def test_resample_matches_oracle(brp, tpl):
    g = _geom(brp)
    rng = np.random.default_rng(1)
    x = rng.normal(7.5, 2.0, g["n_unpadded"]).astype(np.float32)
    out, n_steps, mean = brp.cpu_resample(x, g, *tpl)
    want, ns2, mean2 = reference.resample(x, g, *tpl)
    assert n_steps == ns2
    np.testing.assert_array_equal(out[:n_steps], want[:n_steps])
    assert mean == mean2
    np.testing.assert_allclose(out[n_steps:], mean, rtol=0, atol=0)


def test_power_spectrum_matches_oracle(brp):
    g = _geom(brp)
    rng = np.random.default_rng(2)
    x = rng.normal(0, 1, g["nsamples"]).astype(np.float32)
    ps = brp.cpu_power_spectrum(x, g["fft_size"])
    want = reference.power_spectrum(x, g["fft_size"])
    assert ps[0] == 0.0
    np.testing.assert_allclose(ps, want, rtol=1e-5, atol=1e-6)


def test_harmonic_sum_bitwise(brp):
    g = _geom(brp)
    rng = np.random.default_rng(3)
    ps = rng.exponential(1.0, g["fft_size"]).astype(np.float32)
    # a few strong lines so every level has candidates
    for f in (301, 777, 1203):
        for m in range(1, 17):
            if f * m < g["fft_size"]:
                ps[f * m] += 12.0
    thr = [8.0, 10.0, 14.0, 22.0, 36.0]
    cands, ss = brp.cpu_harmonic_sum(ps, g, thr)
    want = reference.harmonic_sums(ps, g, thr)
    w2 = g["window_2"]
    np.testing.assert_array_equal(ss[:, w2:], want[:, w2:])
    oc = reference.candidates(want, g, thr)
    for h in range(5):
        bins, pw = cands[h]
        np.testing.assert_array_equal(np.asarray(bins), oc[h][0])
        np.testing.assert_array_equal(np.asarray(pw, np.float32), oc[h][1])


def _python_table_apply(table, h, bins, powers, thr, tpl):
    """Literal transcription of the reference insertion loop (one level, one template)."""
    lvl = table[h]
    n_h = 1 << h
    for b, p in zip(bins, powers):
        if p > thr and p > lvl[-1][1]:
            store = len(lvl) - 1
            for k, e in enumerate(lvl):
                if e[0] == b:
                    store = k if e[1] < p else -1
                    break
            if store >= 0:
                lvl[store] = (int(b), float(p), tpl, n_h)
                lvl.sort(key=lambda e: -e[1])


def test_candidate_table_sequential_semantics(brp):
    rng = np.random.default_rng(7)
    t = brp.CandidateTable()
    ref = [[(0, 0.0, None, 0)] * 100 for _ in range(5)]
    chi2 = [5.0, 6.0, 7.0, 8.0, 9.0]
    for n in range(40):
        tpl = (float(np.float32(1000 + n)), float(np.float32(0.01 * n)), float(np.float32(0.1 * n)))
        thr = t.thresholds(chi2)
        for h in range(5):
            # bins from a small pool so that repeated bins (update/keep) occur often
            bins = np.unique(rng.choice(np.arange(50, 450), 60)).astype(np.uint32)
            pw = rng.uniform(0.0, 100.0, bins.size).astype(np.float32)
            sel = pw > thr[h]
            t.apply_level(h, bins[sel], pw[sel], thr[h], *tpl)
            _python_table_apply(ref, h, bins, pw, thr[h], tpl)
    ent = t.entries()
    for h in range(5):
        got = ent[h * 100:(h + 1) * 100]
        for (f0, power, P, tau, psi, nh), (rf0, rp, rtpl, rnh) in zip(got, ref[h]):
            assert f0 == rf0 and power == pytest.approx(rp, rel=0, abs=0)
            if rtpl is not None:
                assert (P, tau, psi) == pytest.approx(rtpl) and nh == rnh


def test_candidate_table_merge_is_exact(brp):
    """Sequential table over templates 0..N == merge of tables over blocks."""
    rng = np.random.default_rng(11)
    chi2 = [5.0, 6.0, 7.0, 8.0, 9.0]
    # per template per level: sorted unique bins and distinct powers
    data = []
    for n in range(60):
        lv = []
        for h in range(5):
            bins = np.unique(rng.choice(np.arange(50, 400), 50)).astype(np.uint32)
            pw = (rng.permutation(bins.size) + rng.uniform(0, 0.5, bins.size) + n * 1e-3 + 10).astype(np.float32)
            lv.append((bins, pw))
        data.append(lv)

    def run(block):
        t = brp.CandidateTable()
        for n in block:
            thr = t.thresholds(chi2)
            tpl = (1000.0 + n, 0.0, 0.0)
            for h in range(5):
                bins, pw = data[n][h]
                sel = pw > thr[h]
                t.apply_level(h, bins[sel], pw[sel], thr[h], *tpl)
        return t

    seq = run(range(60))
    merged = brp.CandidateTable()
    for a, b in ((0, 17), (17, 18), (18, 45), (45, 60)):
        merged.merge(run(range(a, b)))
    assert bytes(seq.to_bytes()) == bytes(merged.to_bytes())


def test_fft_path_any_length(brp):
    """ops.fft_path: smooth lengths take the three-pass FFT, every other
    padding the chirp-z transform over a factorable length >= 2 Mb - 1."""
    from boinc_app_eah_brp_amd import ops

    p = ops.fft_path(3 << 22)
    assert p.kind == "three-pass" and p.dft_len == 3 << 21 and p.work_ratio == 1.0
    for P in (1.1, 1.7, 2.3, 9.9):
        n = int(P * (1 << 22) + 0.5)
        q = ops.fft_path(n)
        assert q.kind == "chirp-z"
        assert q.dft_len == (n if n % 2 else n // 2)
        assert 2 * q.dft_len - 1 <= q.conv_len <= 1.2 * (2 * q.dft_len)
        L1, L2, L3 = q.factors
        assert L1 * L2 * L3 == q.conv_len
    # every padding on a 0.01 grid of [1, 10] at the benchmark's 2^22 samples and at
    # a non-power-of-two sample count has a device plan (odd N up to ~84 M points
    # needs L2 L3 up to 2^18 in the chirp-z convolution)
    for n_u in (1 << 22, 3 * (1 << 20) + 7):
        for k in range(901):
            n = int(float(np.float32(1.0 + 0.01 * k)) * n_u + 0.5)
            assert ops.fft_path(n).kind in ("three-pass", "chirp-z"), n
    # 7-smooth N/2 (radix-7 plan lengths 112 / 224 / 448): the three-pass FFT,
    # not a chirp-z transform over >= 2 Mb - 1 (-P 3.5: N = 7 * 2^21)
    for P, factors in ((3.5, (224, 128, 256)), (6.125, (224, 224, 256))):
        r = ops.fft_path(int(P * (1 << 22) + 0.5))
        assert r.kind == "three-pass" and r.work_ratio == 1.0 and r.factors[:3] == factors, (P, r)
