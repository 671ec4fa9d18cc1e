"""Two-pass vs three-pass FFT plan on the shipped WU (-P 3, the bench geometry).

For a few templates the device power spectrum of each plan (BRP_TWO_PASS=1 /
0, read at engine setup) is compared with the CPU golden model's
double-precision spectrum: largest error relative to max(P_k, mean P) and
where it occurs.

  python tools/two_pass_check.py [--templates 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
WU = ROOT / "data" / "testwu" / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
TEMPLATES = ((1046.6, 0.0547, 4.48), (2000.0, 0.3, 1.0), (11000.0, 0.012, 2.5))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--templates", type=int, default=3)
    a = ap.parse_args()
    from boinc_app_eah_brp_amd import native

    brp = native()
    hdr, series, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=3.0, fA=0.08, window=1000))
    mu = float(np.mean(series))
    engines = {}
    for tp in ("1", "0"):
        os.environ["BRP_TWO_PASS"] = tp  # read at engine setup
        eng = brp.HipEngine()
        eng.init(0, 1)
        eng.setup(geom, series, mu)
        engines[tp] = eng
    out = []
    for P, tau, psi in TEMPLATES[: a.templates]:
        xr, ns_c, _ = brp.cpu_resample(series, geom, P, tau, psi)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        scale = float(np.mean(ps_c[1:]))
        row = dict(P=P, n_steps_cpu=ns_c)
        spectra = {}
        for tp, eng in engines.items():
            ps_g, ns_g = eng.power_spectrum(P, tau, psi)
            spectra[tp] = ps_g.astype(np.float64)
            err = np.abs(spectra[tp] - ps_c)[1:] / np.maximum(ps_c[1:], scale)
            row[f"plan{'2' if tp == '1' else '3'}"] = dict(n_steps=ns_g, max_err=float(err.max()),
                                                          at_bin=int(np.argmax(err)) + 1,
                                                          mean_err=float(err.mean()))
        d = np.abs(spectra["1"] - spectra["0"])[1:] / np.maximum(ps_c[1:], scale)
        row["two_vs_three_max"] = float(d.max())
        out.append(row)
    print(json.dumps(dict(N=int(geom["nsamples"]), results=out)))


if __name__ == "__main__":
    main()
