"""HIP kernels vs the CPU golden model (run on an MI355X: pytest -m gpu)."""
import numpy as np
import pytest

from boinc_app_eah_brp_amd.utils import synth

from conftest import BANK, WU, ZAP

pytestmark = pytest.mark.gpu

OPT_BENCH = dict(f0=400.0, padding=3.0, fA=0.08, window=1000)


def _engine(brp, geom, series, mu0=None, batch=2):
    eng = brp.HipEngine()
    eng.init(0, batch)
    eng.setup(geom, np.ascontiguousarray(series, dtype=np.float32),
              float(np.mean(series)) if mu0 is None else mu0)
    return eng


def _cpu_ps(brp, series, geom, P, tau, psi):
    x, n_steps, mean = brp.cpu_resample(series, geom, P, tau, psi)
    return brp.cpu_power_spectrum(x, geom["fft_size"]), n_steps


@pytest.mark.parametrize("padding", [1.0, 3.0])
def test_power_spectrum_small(brp, gpu, tmp_path, padding):
    case = synth.synthetic_case(tmp_path, n=1 << 16, n_templates=4,
                                inj=synth.Injection(f0=300.0, P_orb=800.0, tau=0.05, psi0=1.0, amplitude=2.0))
    hdr, series, _ = brp.read_work_unit(case["wu"])
    geom = brp.derive_geometry(hdr, dict(OPT_BENCH, padding=padding, f0=200.0, window=100))
    eng = _engine(brp, geom, series)
    for k in range(4):
        P, tau, psi = (np.float32(case[key][k]) for key in ("P", "tau", "psi"))
        ps_gpu, ns_gpu = eng.power_spectrum(float(P), float(tau), float(psi))
        ps_cpu, ns_cpu = _cpu_ps(brp, series, geom, float(P), float(tau), float(psi))
        assert ns_gpu == ns_cpu
        scale = float(np.mean(ps_cpu[1:]))
        err = np.abs(ps_gpu.astype(np.float64) - ps_cpu) / np.maximum(ps_cpu, scale)
        assert err[1:].max() < 2e-4, (k, err.max(), int(np.argmax(err)))


def test_power_spectrum_bench_size(brp, gpu):
    """Benchmark geometry (2^22 samples, P=3 -> 3*2^22-point FFT) on the whitened reference WU."""
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(OPT_BENCH, white=True)
    geom = brp.derive_geometry(hdr, opt)
    eng = _engine(brp, geom, series)
    series = eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
    P, tau, psi = brp.read_template_bank(str(BANK))
    for k in (0, 1):
        ps_gpu, ns_gpu = eng.power_spectrum(float(P[k]), float(tau[k]), float(psi[k]))
        ps_cpu, ns_cpu = _cpu_ps(brp, series, geom, float(P[k]), float(tau[k]), float(psi[k]))
        assert ns_gpu == ns_cpu
        lim = geom["harmonic_idx_hi"]
        scale = float(np.median(ps_cpu[geom["window_2"]:lim]))
        err = np.abs(ps_gpu[1:lim].astype(np.float64) - ps_cpu[1:lim]) / np.maximum(ps_cpu[1:lim], scale)
        assert np.percentile(err, 99.9) < 2e-5, (k, np.percentile(err, 99.9))
        assert err.max() < 1e-3, (k, err.max(), int(np.argmax(err)) + 1)


@pytest.mark.parametrize("full,direct", [("0", "0"), ("0", "1"), ("1", "0")])
@pytest.mark.parametrize("window", [100, 1001, 16, 10, 0])
def test_harmonic_sum_matches_cpu_bitwise(brp, gpu, tmp_path, monkeypatch, window, full, direct):
    """Same power spectrum in -> identical candidate bins and powers out (odd and
    small running-median windows move the first tile's start; below 16 it lies
    before bin 0). Pruned path (bound filter + exact blocks) with LDS-staged
    and with direct bound reads (BRP_HS_DIRECT), and the full gather kernel
    (BRP_HS_FULL=1); the low thresholds flag most blocks."""
    monkeypatch.setenv("BRP_HS_FULL", full)
    monkeypatch.setenv("BRP_HS_DIRECT", direct)
    case = synth.synthetic_case(tmp_path, n=1 << 17, n_templates=2,
                                inj=synth.Injection(f0=150.0, P_orb=900.0, tau=0.02, psi0=2.0, amplitude=3.0))
    hdr, series, _ = brp.read_work_unit(case["wu"])
    geom = brp.derive_geometry(hdr, dict(f0=120.0, padding=3.0, fA=0.08, window=window))
    eng = _engine(brp, geom, series, batch=1)
    P, tau, psi = (np.float32(case[key][0]) for key in ("P", "tau", "psi"))
    thr = [4.0, 6.0, 9.0, 14.0, 24.0]  # low thresholds -> many candidates
    out = eng.process(np.array([P]), np.array([tau]), np.array([psi]), thr)[0]
    ps_gpu, _ = eng.power_spectrum(float(P), float(tau), float(psi))
    ref, _ = brp.cpu_harmonic_sum(ps_gpu, geom, thr)
    for h in range(5):
        bins_g, pw_g = out[h]
        bins_c, pw_c = ref[h]
        assert len(bins_c) > 0
        np.testing.assert_array_equal(bins_g, bins_c)
        np.testing.assert_array_equal(pw_g, pw_c)


@pytest.mark.parametrize("full,thr,cell,direct", [("0", (9.0, 12.0, 16.0, 22.0, 33.0), "8", "0"),
                                                  ("0", (9.0, 12.0, 16.0, 22.0, 33.0), "8", "1"),
                                                  ("1", (9.0, 12.0, 16.0, 22.0, 33.0), "8", "0"),
                                                  ("0", (11.0, 12.5, 15.5, 21.0, 31.0), "8", "0"),
                                                  ("0", (11.0, 12.5, 15.5, 21.0, 31.0), "8", "1"),
                                                  ("0", (13.0, 15.0, 18.0, 24.0, 34.5), "8", "0"),
                                                  ("0", (13.0, 15.0, 18.0, 24.0, 34.5), "8", "1"),
                                                  ("0", (11.0, 12.5, 15.5, 21.0, 31.0), "4", "0"),
                                                  ("0", (18.139, 21.241, 26.269, 34.648, 48.958), "8", "0"),
                                                  ("0", (18.139, 21.241, 26.269, 34.648, 48.958), "8", "1")])
def test_harmonic_sum_bench_size_matches_cpu_bitwise(brp, gpu, monkeypatch, full, thr, cell, direct):
    """Benchmark geometry (hhi = 5.27 M bins, two templates of a batch): the
    harmonic-sum candidates equal the CPU model's on the same spectrum, for the
    pruned path at thresholds that flag many / some / few blocks (down to the
    search's chi^2 levels), with 8-bin and 4-bin bound cells, LDS-staged and
    direct bound reads (BRP_HS_DIRECT), and for the full gather kernel."""
    monkeypatch.setenv("BRP_HS_FULL", full)
    monkeypatch.setenv("BRP_HS_CELL", cell)
    monkeypatch.setenv("BRP_HS_DIRECT", direct)
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(OPT_BENCH, white=True)
    geom = brp.derive_geometry(hdr, opt)
    eng = _engine(brp, geom, series, batch=2)
    series = eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
    P, tau, psi = brp.read_template_bank(str(BANK))
    thr = list(thr)
    outs = eng.process(P[:2].astype(np.float32), tau[:2].astype(np.float32), psi[:2].astype(np.float32), thr)
    for k in range(2):
        ps_gpu, _ = eng.power_spectrum(float(np.float32(P[k])), float(np.float32(tau[k])), float(np.float32(psi[k])))
        ref, _ = brp.cpu_harmonic_sum(ps_gpu, geom, thr)
        assert sum(len(ref[h][0]) for h in range(5)) > 0 or thr[0] > 18.0
        for h in range(5):
            assert len(ref[h][0]) > 0 or thr[0] > 10.0
            np.testing.assert_array_equal(outs[k][h][0], ref[h][0])
            np.testing.assert_array_equal(outs[k][h][1], ref[h][1])


def _host_cells(ps, geom, n):
    """8-bin maxima of the stored spectrum (bins < min(hhi, fft_size)), zero beyond"""
    lim = min(geom["harmonic_idx_hi"], geom["fft_size"])
    v = np.zeros(8 * n, np.float32)
    m = min(lim, 8 * n, len(ps))
    v[:m] = ps[:m]
    return v.reshape(n, 8).max(axis=1)


@pytest.mark.parametrize("cells", ["hs_cells", "hs_cells8", "p3"])
@pytest.mark.parametrize("case", ["bench", "small"])
def test_bound_cells_equal_spectrum_maxima(brp, gpu, tmp_path, monkeypatch, case, cells):
    """The pruned harmonic sum's 8-bin bound cells (hs_cells_kernel; 4 cells
    per thread with BRP_HS_CELLS_CPT=4; with BRP_P3_CELLS=1 the own-bin cells
    from pass 3 and the mirror half from hs_cells_kernel) equal the 8-bin
    maxima of the spectrum pass 3 stored, bit for bit, zero beyond the harmonic
    range (the bounds' monotonicity argument needs cells >= every bin)."""
    monkeypatch.setenv("BRP_P3_CELLS", "1" if cells == "p3" else "0")
    monkeypatch.setenv("BRP_HS_CELLS_CPT", "4" if cells == "hs_cells8" else "1")
    opt = None
    if case == "bench":
        hdr, series, _ = brp.read_work_unit(str(WU))
        opt = dict(OPT_BENCH, white=True)
        geom = brp.derive_geometry(hdr, opt)
        P, tau, psi = brp.read_template_bank(str(BANK))
        P, tau, psi = P[:2], tau[:2], psi[:2]
    else:
        c = synth.synthetic_case(tmp_path, n=1 << 17, n_templates=2,
                                 inj=synth.Injection(f0=150.0, P_orb=900.0, tau=0.02, psi0=2.0, amplitude=3.0))
        hdr, series, _ = brp.read_work_unit(c["wu"])
        geom = brp.derive_geometry(hdr, dict(f0=120.0, padding=3.0, fA=0.08, window=100))
        P, tau, psi = (np.asarray(c[key][:2]) for key in ("P", "tau", "psi"))
    eng = _engine(brp, geom, series, batch=2)
    if opt is not None:  # the benchmark WU is searched whitened
        eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
    eng.process(P.astype(np.float32), tau.astype(np.float32), psi.astype(np.float32),
                [18.139, 21.241, 26.269, 34.648, 48.958])
    cells = [eng.bound_cells(k) for k in range(2)]
    for k in range(2):
        ps, _ = eng.power_spectrum(float(np.float32(P[k])), float(np.float32(tau[k])), float(np.float32(psi[k])))
        np.testing.assert_array_equal(cells[k], _host_cells(np.asarray(ps), geom, len(cells[k])))


@pytest.mark.parametrize("thr", [(9.0, 12.0, 16.0, 22.0, 33.0), (18.139, 21.241, 26.269, 34.648, 48.958)])
def test_harmonic_sum_fp16_pruned_equals_full(brp, gpu, monkeypatch, thr):
    """Config 5 (fp16 spectrum): the pruned harmonic sum (bounds from fp32 cell
    maxima of the fp16 spectrum, exact sums widened to fp32) gives the
    candidate lists of the full fp16 gather kernel bit for bit, on the
    benchmark geometry."""
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(OPT_BENCH, white=True)
    geom = brp.derive_geometry(hdr, opt)
    P, tau, psi = brp.read_template_bank(str(BANK))
    outs = {}
    for full, direct in (("0", "0"), ("1", "0"), ("d", "1")):
        monkeypatch.setenv("BRP_HS_FULL", "1" if full == "1" else "0")
        monkeypatch.setenv("BRP_HS_DIRECT", direct)
        eng = _engine(brp, geom, series, batch=2)
        eng.set_ps_fp16(True)
        eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
        outs[full] = eng.process(P[:2].astype(np.float32), tau[:2].astype(np.float32), psi[:2].astype(np.float32),
                                 list(thr))
    assert sum(len(outs["1"][k][h][0]) for k in range(2) for h in range(5)) > 0 or thr[0] > 18.0
    for k in range(2):
        for h in range(5):
            for v in ("0", "d"):  # LDS-staged and direct bound reads
                np.testing.assert_array_equal(outs[v][k][h][0], outs["1"][k][h][0])
                np.testing.assert_array_equal(outs[v][k][h][1], outs["1"][k][h][1])


def test_engine_batches_in_flight_match_process(brp, gpu):
    """Pipelined engine API: max_in_flight() batches submitted back to back
    (double-buffered parameters and candidate lists, one stream) complete in
    submission order with the candidates process() gives one batch at a time;
    process() refuses to run while batches are outstanding."""
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(OPT_BENCH, white=True)
    geom = brp.derive_geometry(hdr, opt)
    eng = _engine(brp, geom, series, batch=1)
    eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
    P, tau, psi = (x.astype(np.float32) for x in brp.read_template_bank(str(BANK)))
    thr = [9.0, 12.0, 16.0, 22.0, 33.0]
    depth = eng.max_in_flight()
    assert depth >= 2
    ref = [eng.process(P[k:k + 1], tau[k:k + 1], psi[k:k + 1], thr)[0] for k in range(depth + 1)]
    for k in range(depth):
        eng.submit(P[k:k + 1], tau[k:k + 1], psi[k:k + 1], thr)
    with pytest.raises(Exception):
        eng.process(P[:1], tau[:1], psi[:1], thr)
    got = [eng.complete()[0]]
    eng.submit(P[depth:depth + 1], tau[depth:depth + 1], psi[depth:depth + 1], thr)  # reuses a completed slot
    got += [eng.complete()[0] for _ in range(depth)]
    assert sum(len(ref[k][h][0]) for k in range(depth + 1) for h in range(5)) > 0
    for k in range(depth + 1):
        for h in range(5):
            np.testing.assert_array_equal(got[k][h][0], ref[k][h][0])
            np.testing.assert_array_equal(got[k][h][1], ref[k][h][1])
    with pytest.raises(Exception):
        eng.complete()  # nothing outstanding


@pytest.mark.parametrize("batch,serial", [(1, 4), (2, 3), (1, 8)])
def test_serial_launch_groups_match_single_templates(brp, gpu, monkeypatch, batch, serial):
    """Serial launch groups (BRP_SERIAL): one submitted batch of batch x serial
    templates runs its launch groups back to back through the same FFT buffers
    into one candidate list (keys offset by the group's first template). Every
    template's candidates equal those of one-template batches, bit for bit,
    including a short last group."""
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(OPT_BENCH, white=True)
    geom = brp.derive_geometry(hdr, opt)
    P, tau, psi = (x.astype(np.float32) for x in brp.read_template_bank(str(BANK)))
    thr = [9.0, 12.0, 16.0, 22.0, 33.0]
    n = batch * serial - 1  # the last launch group is short when batch > 1
    monkeypatch.setenv("BRP_SERIAL", "1")
    one = _engine(brp, geom, series, batch=1)
    one.whiten(opt, brp.read_zaplist(str(ZAP)), series.copy())
    assert one.batch() == 1
    ref = [one.process(P[k:k + 1], tau[k:k + 1], psi[k:k + 1], thr)[0] for k in range(n)]
    monkeypatch.setenv("BRP_SERIAL", str(serial))
    grp = _engine(brp, geom, series, batch=batch)
    grp.whiten(opt, brp.read_zaplist(str(ZAP)), series.copy())
    assert grp.batch() == batch * serial
    got = grp.process(P[:n], tau[:n], psi[:n], thr)
    assert sum(len(ref[k][h][0]) for k in range(n) for h in range(5)) > 0
    for k in range(n):
        for h in range(5):
            np.testing.assert_array_equal(got[k][h][0], ref[k][h][0])
            np.testing.assert_array_equal(got[k][h][1], ref[k][h][1])


def test_whitening_wide_window_matches_cpu(brp, gpu, tmp_path):
    """-B above the LDS kernel's 3072: whitening stays on the device (wide
    running median) and matches the CPU whitening."""
    case = synth.synthetic_case(tmp_path, n=1 << 16, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    opt = dict(f0=200.0, padding=3.0, fA=0.08, window=5001, white=True)
    geom = brp.derive_geometry(hdr, opt)
    zaps = brp.read_zaplist(case["zap"])
    w_cpu = brp.cpu_whiten(series, geom, opt, zaps)
    eng = _engine(brp, geom, series)
    w_gpu = eng.whiten(opt, zaps, series)
    rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
    assert rms > 0
    assert np.max(np.abs(w_gpu - w_cpu)) / rms < 1e-4


def test_whitening_matches_cpu(brp, gpu, tmp_path):
    case = synth.synthetic_case(tmp_path, n=1 << 16, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    opt = dict(f0=200.0, padding=3.0, fA=0.08, window=200, white=True)
    geom = brp.derive_geometry(hdr, opt)
    zaps = brp.read_zaplist(case["zap"])
    w_cpu = brp.cpu_whiten(series, geom, opt, zaps)
    eng = _engine(brp, geom, series)
    w_gpu = eng.whiten(opt, zaps, series)
    rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
    assert rms > 0
    assert np.max(np.abs(w_gpu - w_cpu)) / rms < 1e-4


def test_running_median_gpu_exact(brp, gpu, tmp_path):
    """The device running median must be bit-identical to the host one (via whitening scale)."""
    case = synth.synthetic_case(tmp_path, n=1 << 15, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    for window in (99, 100, 1000):
        opt = dict(f0=200.0, padding=1.0, fA=0.08, window=window, white=True)
        geom = brp.derive_geometry(hdr, opt)
        w_cpu = brp.cpu_whiten(series, geom, opt, [])
        eng = _engine(brp, geom, series)
        w_gpu = eng.whiten(opt, [], series)
        rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
        assert np.max(np.abs(w_gpu - w_cpu)) / rms < 1e-4, window


def test_whitening_overlapping_zaps_deterministic(brp, gpu, tmp_path):
    """Overlapping zap ranges hit bins several times; the sequential reference
    keeps the last draw. The device result must match the CPU and be identical
    run to run (a parallel write of duplicates would race)."""
    case = synth.synthetic_case(tmp_path, n=1 << 16, n_templates=1)
    hdr, series, _ = brp.read_work_unit(case["wu"])
    opt = dict(f0=200.0, padding=3.0, fA=0.08, window=200, white=True)
    geom = brp.derive_geometry(hdr, opt)
    zaps = [(10.0, 12.0), (11.0, 13.0), (11.5, 11.6), (50.0, 50.5), (49.9, 50.2)]
    w_cpu = brp.cpu_whiten(series, geom, opt, zaps)
    eng = _engine(brp, geom, series)
    w1 = eng.whiten(opt, zaps, series)
    eng.setup(geom, np.ascontiguousarray(series, dtype=np.float32), float(np.mean(series)))
    w2 = eng.whiten(opt, zaps, series)
    np.testing.assert_array_equal(w1, w2)
    rms = float(np.sqrt(np.mean(w_cpu.astype(np.float64) ** 2)))
    assert np.max(np.abs(w1 - w_cpu)) / rms < 1e-4


@pytest.mark.parametrize("w", [1, 2, 99, 100, 1000, 3072, 3073, 4096, 10001, 12288, 12289, 65536, 250000])
def test_running_median_kernel_bit_exact(brp, gpu, w):
    """Device running median == host running median, bit for bit, with ties.
    Windows above 3072 take the wide path (global radix sort + median walk,
    rmed_wide.hip) up to the reference's limit of 250 000."""
    rng = np.random.default_rng(w)
    n = 50_000 + 3 * w if w <= 3072 else w + 30_000
    x = rng.exponential(size=n).astype(np.float32)
    x[::7] = np.round(x[::7], 1)  # many exact ties
    x[100:400] = 0.25  # a run of equal values
    ref = brp.running_median(x, w)
    got, _ = brp.hip_running_median(x, w)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("four_bit", [True, False])
def test_device_unpack_bit_exact(brp, gpu, tmp_path, four_bit):
    """The device unpacks the WU payload (HipEngine.setup_packed: n/2 bytes over
    PCIe instead of 4n) to exactly the floats of the host reader
    (io.cpp, demod_binary.c:830-842): 4-bit high nibble first, 8-bit signed,
    value / scale in double. Odd sample count included."""
    from boinc_app_eah_brp_amd.utils import synth

    x = synth.make_series((1 << 14) + 1, 65.476, None)
    wu = synth.write_wu(tmp_path / ("a.bin4" if four_bit else "a.binary"), x, four_bit=four_bit, scale=0.37)
    hdr, series, _ = brp.read_work_unit(str(wu))
    geom = brp.derive_geometry(hdr, dict(f0=150.0, padding=2.0, fA=0.08, window=100))
    eng = brp.HipEngine()
    eng.init(0, 1)
    eng.setup_from_wu(geom, str(wu), 0.0)
    dev = eng.download_series()
    assert dev.dtype == np.float32 and dev.size == series.size
    assert np.array_equal(dev.view(np.uint32), np.asarray(series, np.float32).view(np.uint32))
