"""Child process of tests/test_gpu_checked.py: the benchmark geometry's
whitened 2-template batch through the CHECKED build (BRP_CHECKED=1 selects the
module _brp_checked; csrc/hip/checked.hpp), then the test hooks and a
device check. Prints one JSON line: whether process() raised, the messages,
and whether the device check was clean.

usage: python tests/_checked_run.py [--hooks]
(BRP_CHECKED_INJECT=<site> in the environment injects one out-of-bounds access)
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ["BRP_CHECKED"] = "1"

import numpy as np  # noqa: E402

import boinc_app_eah_brp_amd as pkg  # noqa: E402

DATA = ROOT / "data" / "testwu"
WU = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
BANK = DATA / "stochastic_full.bank"
ZAP = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"


def main() -> int:
    brp = pkg.native()
    out = {"checked": bool(brp.checked_build()), "process_error": None, "hooks_error": None, "device_check": None,
           "n_cands": 0, "cells_ok": None}
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
    geom = brp.derive_geometry(hdr, opt)
    P, tau, psi = (x[:2].astype(np.float32) for x in brp.read_template_bank(str(BANK)))
    eng = brp.HipEngine()
    eng.init(0, 2)
    eng.setup(geom, np.ascontiguousarray(series, dtype=np.float32), float(np.mean(series)))
    eng.whiten(opt, brp.read_zaplist(str(ZAP)), series)
    try:
        res = eng.process(P, tau, psi, [18.139, 21.241, 26.269, 34.648, 48.958])
        out["n_cands"] = int(sum(len(res[k][h][0]) for k in range(2) for h in range(5)))
    except RuntimeError as e:
        out["process_error"] = str(e)
    if "--hooks" in sys.argv and out["process_error"] is None:
        try:
            cells = eng.bound_cells(0)
            ps, _ = eng.power_spectrum(float(P[0]), float(tau[0]), float(psi[0]))
            lim = min(geom["harmonic_idx_hi"], geom["fft_size"])
            v = np.zeros(8 * len(cells), np.float32)
            m = min(lim, 8 * len(cells), len(ps))
            v[:m] = ps[:m]
            out["cells_ok"] = bool(np.array_equal(cells, v.reshape(-1, 8).max(axis=1)))
            eng.download_series()
        except RuntimeError as e:
            out["hooks_error"] = str(e)
    try:
        brp.device_check()
        out["device_check"] = "clean"
    except RuntimeError as e:
        out["device_check"] = str(e)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
