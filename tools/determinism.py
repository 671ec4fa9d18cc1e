"""Run-to-run determinism checks on the GPU (benchmark WU):
whitening, single-template power spectra, and full-search candidate tables
with one and two pipelines per device."""
import json
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import boinc_app_eah_brp_amd as pkg  # noqa: E402
from boinc_app_eah_brp_amd.parallel import DistContext, ShardedSearch  # noqa: E402

D = Path(__file__).resolve().parent.parent / "data" / "testwu"
WU = D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
BANK = D / "stochastic_full.bank"
ZAP = D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"
brp = pkg.native()
brp.set_log_level(2)
out = {}
hdr, series, _ = brp.read_work_unit(str(WU))
opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
geom = brp.derive_geometry(hdr, opt)
zaps = brp.read_zaplist(str(ZAP))
eng = brp.HipEngine()
eng.init(0, 4)
eng.setup(geom, series, float(np.mean(series)))
w1 = eng.whiten(opt, zaps, series)
eng.setup(geom, series, float(np.mean(series)))
w2 = eng.whiten(opt, zaps, series)
out["whiten_identical"] = bool(np.array_equal(w1, w2))
P, tau, psi = brp.read_template_bank(str(BANK))
same = True
for k in (0, 5, 17):
    a, _ = eng.power_spectrum(float(P[k]), float(tau[k]), float(psi[k]))
    b, _ = eng.power_spectrum(float(P[k]), float(tau[k]), float(psi[k]))
    same &= bool(np.array_equal(a, b))
out["ps_identical"] = same
n = int(sys.argv[1]) if len(sys.argv) > 1 else 800
opts = dict(inputfile=str(WU), templatebank=str(BANK), zaplistfile=str(ZAP), f0=400.0, padding=3.0, fA=0.08,
            window=1000, white=True, batch=8)
for streams in (1, 2):
    ss = ShardedSearch(opts, DistContext(), streams=streams)
    t1 = bytes(ss.step(n).to_bytes())
    t2 = bytes(ss.step(n).to_bytes())
    out[f"table_identical_streams{streams}"] = t1 == t2
    out[f"table_s{streams}"] = t1
out["table_streams1_vs_2"] = out.pop("table_s1") == out.pop("table_s2")
print(json.dumps(out))
