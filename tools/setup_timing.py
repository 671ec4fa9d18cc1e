"""Host-side cost of bringing up HIP pipelines for the benchmark WU (GPU)."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import boinc_app_eah_brp_amd as pkg  # noqa: E402

D = Path(__file__).resolve().parent.parent / "data" / "testwu"
brp = pkg.native()
brp.set_log_level(2)
t = time.perf_counter()
hdr, series, _ = brp.read_work_unit(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"))
print(f"read WU {1e3 * (time.perf_counter() - t):.1f} ms")
opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
geom = brp.derive_geometry(hdr, opt)
engs = []
for k in range(3):
    t = time.perf_counter()
    e = brp.HipEngine()
    e.init(0, 1)
    t1 = time.perf_counter()
    e.setup(geom, series, float(np.mean(series)))
    t2 = time.perf_counter()
    print(f"engine {k}: init {1e3 * (t1 - t):.1f} ms  setup {1e3 * (t2 - t1):.1f} ms")
    engs.append(e)
t = time.perf_counter()
w = engs[0].whiten(opt, brp.read_zaplist(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap")), series)
print(f"whiten {1e3 * (time.perf_counter() - t):.1f} ms")
t = time.perf_counter()
engs[1].setup(geom, w, 0.0)
print(f"same-shape re-setup {1e3 * (time.perf_counter() - t):.1f} ms")
