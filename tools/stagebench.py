"""Per-stage timing of the template pipeline on the benchmark WU (GPU)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import boinc_app_eah_brp_amd as pkg  # noqa: E402

D = Path(__file__).resolve().parent.parent / "data" / "testwu"
brp = pkg.native()
brp.set_log_level(2)
hdr, series, _ = brp.read_work_unit(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"))
opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
geom = brp.derive_geometry(hdr, opt)
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 4
eng = brp.HipEngine()
eng.init(0, batch)
eng.setup(geom, series, float(np.mean(series)))
w = eng.whiten(opt, brp.read_zaplist(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap")), series)
P, tau, psi = brp.read_template_bank(str(D / "stochastic_full.bank"))
res = eng.benchmark_stages(P[:batch].astype(np.float32), tau[:batch].astype(np.float32), psi[:batch].astype(np.float32), 20)
res = {k: round(v / batch, 2) for k, v in res.items()}
print(json.dumps({"us_per_template": res, "batch": batch, "plan": eng.plan()}))
