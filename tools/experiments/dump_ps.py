"""Dump the power spectrum of one benchmark template (whitened reference WU,
-P 3 -f 400 -A 0.08 -W) for tools/experiments/hs_variants; prints the
geometry arguments the harness needs."""
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import boinc_app_eah_brp_amd as pkg  # noqa: E402

D = ROOT / "data" / "testwu"
brp = pkg.native()
brp.set_log_level(2)
hdr, series, _ = brp.read_work_unit(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"))
opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
g = brp.derive_geometry(hdr, opt)
eng = brp.HipEngine()
eng.init(0, 1)
eng.setup(g, series, float(np.mean(series)))
series = eng.whiten(opt, brp.read_zaplist(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap")), series)
P, tau, psi = brp.read_template_bank(str(D / "stochastic_full.bank"))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ps, _ = eng.power_spectrum(float(np.float32(P[k])), float(np.float32(tau[k])), float(np.float32(psi[k])))
ps.astype(np.float32).tofile(sys.argv[1])
print(g["window_2"], g["fundamental_idx_hi"], min(g["harmonic_idx_hi"], g["fft_size"]))
