"""Time the device running median at the whitening shape of the benchmark WU
(fft_size bins, window 1000): python tools/rmed_bench.py [n] [w] [reps]."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import boinc_app_eah_brp_amd as pkg  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6291457
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    brp = pkg.native()
    x = np.random.default_rng(0).exponential(size=n).astype(np.float32)
    out, ms = brp.hip_running_median(x, w, reps)
    t = time.perf_counter()
    ref = brp.running_median(x, w)
    cpu_ms = 1e3 * (time.perf_counter() - t)
    print(f"n={n} w={w}: device {ms:.3f} ms/call, host {cpu_ms:.1f} ms, exact={np.array_equal(out, ref)}")


if __name__ == "__main__":
    main()
