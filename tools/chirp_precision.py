"""Chirp-z (Bluestein) spectrum precision at production size on the GPU.

For the shipped 2^22-sample WU at a padding outside the three-pass set, the
device power spectrum of a few templates is compared with the CPU golden
model's double-precision spectrum: the largest error relative to
max(P_k, mean P), where it occurs, and the same over bins >= 1000.

  python tools/chirp_precision.py [--padding 2.7] [--so path/to/_brp*.so]

--so loads another build of the native module (A/B of two builds in one call).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
WU = ROOT / "data" / "testwu" / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"


def load(so: str | None):
    if not so:
        from boinc_app_eah_brp_amd import native

        return native()
    spec = importlib.util.spec_from_file_location("_brp", so)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--padding", type=float, default=2.7)
    ap.add_argument("--so", default="")
    ap.add_argument("--templates", type=int, default=2)
    a = ap.parse_args()
    brp = load(a.so)
    hdr, series, _ = brp.read_work_unit(str(WU))
    geom = brp.derive_geometry(hdr, dict(f0=400.0, padding=a.padding, fA=0.08, window=1000))
    eng = brp.HipEngine()
    eng.init(0, 1)
    eng.setup(geom, series, float(np.mean(series)))
    out = []
    for P, tau, psi in ((1046.6, 0.0547, 4.48), (2000.0, 0.3, 1.0))[: a.templates]:
        ps_g, ns_g = eng.power_spectrum(P, tau, psi)
        xr, ns_c, _ = brp.cpu_resample(series, geom, P, tau, psi)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        scale = float(np.mean(ps_c[1:]))
        err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
        hi = err[999:]
        out.append(dict(P=P, n_steps=(ns_g, ns_c), max_err=float(err.max()), at_bin=int(np.argmax(err)) + 1,
                        max_err_bins_ge_1000=float(hi.max()), first_bins_err=[float(x) for x in err[:4]],
                        first_bins_gpu=[float(x) for x in ps_g[1:5]], first_bins_cpu=[float(x) for x in ps_c[1:5]]))
    print(json.dumps(dict(so=a.so or "tree", N=int(geom["nsamples"]), results=out)))


if __name__ == "__main__":
    main()
