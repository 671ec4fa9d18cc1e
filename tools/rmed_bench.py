"""Device running-median timing on the whitening shape (6.29 M bins, W = 1000)
and a bit-exactness check against the host median; run once per BRP_RMED_*
setting (the launcher reads the switch once per process)."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from boinc_app_eah_brp_amd import native  # noqa: E402

brp = native()
rng = np.random.default_rng(1)
n, w = 6291456, 1000
x = rng.exponential(size=n).astype(np.float32)
x[::7] = np.round(x[::7], 1)
got, ms = brp.hip_running_median(x, w, 20)
ref = brp.running_median(x[:400000], w)
ok = np.array_equal(got[:ref.size], ref)
print(f"rmed {os.environ.get('BRP_RMED_REG', '0')} W={w} n={n}: {ms * 1e3:.1f} us per call, exact on the first 400k: {ok}")
