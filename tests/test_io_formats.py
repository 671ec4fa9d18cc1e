"""File formats and I/O (reference structs.h, demod_binary.c:300-760, 1590-1690).

The benchmark work unit, template bank and zaplist under data/testwu are the
files shipped with the reference; everything else is written by our own
writers and read back."""
import math

import numpy as np
import pytest

from conftest import BANK, WU, ZAP


def test_struct_sizes(brp):
    # packed on-disk layouts of structs.h: header 1168 B, checkpoint header 260 B, candidate 48 B
    assert brp.DD_HEADER_SIZE == 1168
    assert brp.CP_HEADER_SIZE == 260
    assert brp.CP_CAND_SIZE == 48
    assert brp.N_CAND == 500 and brp.N_CAND_5 == 100


def test_read_shipped_work_unit(brp):
    hdr, s, four_bit = brp.read_work_unit(str(WU))
    assert four_bit
    assert hdr["nsamples"] == 1 << 22 and s.shape == (1 << 22,)
    assert math.isclose(hdr["tsample"], 65.476190476, rel_tol=1e-9)
    assert math.isclose(hdr["DM"], 109.9)
    assert hdr["name"] == "G187.41-00.88.N"
    # 4-bit payload dequantised as nibble / scale: every sample is k / scale, k in 0..15
    k = s.astype(np.float64) * hdr["scale"]
    assert np.all(np.abs(k - np.rint(k)) < 1e-3)
    assert k.min() >= -1e-3 and k.max() <= 15 + 1e-3


@pytest.mark.parametrize("four_bit", [True, False])
@pytest.mark.parametrize("gz", [True, False])
def test_work_unit_roundtrip(brp, tmp_path, four_bit, gz):
    from boinc_app_eah_brp_amd.utils import synth

    x = synth.make_series(4096, 65.476, seed=3)
    # the format is chosen by extension: ".bin4" 4-bit, ".binary" 8-bit (demod_binary.c:315-327)
    p = synth.write_wu(tmp_path / ("wu.bin4" if four_bit else "wu.binary"), x, four_bit=four_bit, gzip=gz, scale=2.0, name="RT")
    hdr, s, fb = brp.read_work_unit(str(p))
    assert fb == four_bit and hdr["name"] == "RT" and hdr["nsamples"] == 4096
    if four_bit:
        want = np.clip(np.rint(x), 0, 15) / 2.0
    else:
        want = np.clip(np.rint((x - 7.5) * 8.0), -128, 127) / 2.0
    np.testing.assert_allclose(s, want.astype(np.float32), rtol=0, atol=1e-6)


def test_read_template_bank(brp):
    P, tau, psi = brp.read_template_bank(str(BANK))
    assert len(P) == len(tau) == len(psi) == 6662
    # first template of the shipped bank is the unmodulated one
    assert (P[0], tau[0], psi[0]) == (1000.0, 0.0, 0.0)
    assert np.all((P[1:] > 600) & (P[1:] < 2300)) and np.all((tau >= 0) & (tau < 0.4))


def test_bank_trailing_line_quirk(brp, tmp_path):
    # the reference loop `while(fgets(...) && !feof(...))` drops a final line
    # without newline; a final line with newline is kept
    p = tmp_path / "b.bank"
    p.write_text("1000 0 0\n1100 0.1 0.2\n1200 0.2 0.3")
    assert len(brp.read_template_bank(str(p))[0]) == 2
    p.write_text("1000 0 0\n1100 0.1 0.2\n1200 0.2 0.3\n")
    assert len(brp.read_template_bank(str(p))[0]) == 3


def test_read_zaplist(brp):
    z = brp.read_zaplist(str(ZAP))
    assert z[0] == (59.9, 60.1) and len(z) > 10
    assert all(lo <= hi for lo, hi in z)


def test_checkpoint_roundtrip(brp, tmp_path):
    t = brp.CandidateTable()
    rng = np.random.default_rng(0)
    for h in range(5):
        bins = np.sort(rng.choice(np.arange(100, 10000), 30, replace=False)).astype(np.uint32)
        pw = rng.uniform(50, 100, 30).astype(np.float32)
        t.apply_level(h, bins, pw, 20.0, 1000.0 + h, 0.1, 0.2)
    p = tmp_path / "cp.cpt"
    brp.write_checkpoint(str(p), 1234, "orig.bin4", t)
    assert p.stat().st_size == 260 + 500 * 48
    n, orig, t2 = brp.read_checkpoint(str(p))
    assert n == 1234 and orig == "orig.bin4"
    assert bytes(t.to_bytes()) == bytes(t2.to_bytes())
    assert brp.read_checkpoint(str(tmp_path / "missing.cpt")) is None


def test_results_file_format(brp, tmp_path):
    t = brp.CandidateTable()
    # two levels, one shared f0 bin: the result file keeps one line per f0
    t.apply_level(0, np.array([1000, 2000], np.uint32), np.array([40.0, 60.0], np.float32), 20.0, 1000.0, 0.1, 0.2)
    t.apply_level(3, np.array([2000, 3000], np.uint32), np.array([90.0, 95.0], np.float32), 30.0, 1100.0, 0.2, 0.3)
    p = tmp_path / "res.cand"
    t_obs = 823.88
    brp.write_results(str(p), t, t_obs, False)
    lines, done = brp.read_results(str(p))
    assert done
    text = p.read_text().splitlines()
    assert text[-1] == "%DONE%"
    f0s = [l[0] for l in lines]
    assert len(f0s) == len(set(f0s)) == 3
    # frequency = bin / t_obs
    assert set(round(f * t_obs) for f in f0s) == {1000, 2000, 3000}
    for f, P, tau, psi, power, fa, nh in lines:
        assert nh in (1, 8) and power > 0 and fa >= 0
