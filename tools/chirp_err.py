"""Max relative spectrum error of the device chirp-z / three-pass FFT against
the CPU double model for a few (samples, padding) cases (GPU; diagnostics).

  python tools/chirp_err.py"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("BRP_CPU_MEAN", "double")
import boinc_app_eah_brp_amd as pkg  # noqa: E402
from boinc_app_eah_brp_amd.utils import synth  # noqa: E402

INJ = synth.Injection(f0=97.0, P_orb=700.0, tau=0.02, psi0=0.3, amplitude=2.0)
CASES = [(1 << 21, 7.01), (1 << 21, 5.02), (1 << 21, 6.14), (1 << 21, 7.89), (1 << 20, 7.88), (1 << 20, 6.13)]


def main():
    cases = [tuple(float(v) if "." in v else int(v) for v in c.split(":")) for c in os.environ.get("CASES", "").split()] or CASES
    brp = pkg.native()
    d = Path(tempfile.mkdtemp())
    for n, P in cases:
        x = synth.make_series(n, 65.476, INJ)
        wu = synth.write_wu(d / "a.bin4", x)
        hdr, series, _ = brp.read_work_unit(str(wu))
        geom = brp.derive_geometry(hdr, dict(f0=150.0, padding=P, fA=0.08, window=100))
        eng = brp.HipEngine()
        eng.init(0, 2)
        eng.setup(geom, series, float(np.mean(series)))
        ps_g, _ = eng.power_spectrum(900.0, 0.05, 1.3)
        xr, _, _ = brp.cpu_resample(series, geom, 900.0, 0.05, 1.3)
        ps_c = brp.cpu_power_spectrum(xr, geom["fft_size"])
        scale = float(np.mean(ps_c[1:]))
        err = np.abs(ps_g.astype(np.float64) - ps_c)[1:] / np.maximum(ps_c[1:], scale)
        N = geom["nsamples"]
        print(f"n={n} P={P} N={N} plan={brp.bluestein_plan(N if N % 2 else N // 2)} "
              f"max={err.max():.3e} p99.99={np.quantile(err, 0.9999):.3e} mean={err.mean():.3e}", flush=True)
        if os.environ.get("DETAIL"):
            top = np.argsort(err)[-8:][::-1]
            print("  top bins:", " ".join(f"{int(i) + 1}:{err[i]:.2e}" for i in top), flush=True)
            dec = np.array_split(err, 16)
            print("  mean by 16ths:", " ".join(f"{d.mean():.2e}" for d in dec), flush=True)
            print("  max by 16ths:", " ".join(f"{d.max():.1e}" for d in dec), flush=True)


if __name__ == "__main__":
    main()
