"""Time the device running median at the whitening shape of the benchmark WU
(fft_size = 6 291 457 bins): python tools/rmed_bench.py [--n N] [--reps R] W [W ...].
Windows up to 3072 use the LDS kernel, wider ones the radix-sort median walk
(csrc/hip/rmed_wide.hip). The host reference is timed and compared only where
it is affordable (its sorted-window update moves O(W) bytes per output)."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import boinc_app_eah_brp_amd as pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("windows", nargs="*", type=int, default=[1000])
    ap.add_argument("--n", type=int, default=6291457)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host-limit", type=int, default=3072, help="compare with the host for W <= this")
    args = ap.parse_args()
    brp = pkg.native()
    x = np.random.default_rng(0).exponential(size=args.n).astype(np.float32)
    for w in args.windows:
        out, ms = brp.hip_running_median(x, w, args.reps)
        line = f"n={args.n} w={w}: device {ms:.3f} ms/call"
        if w <= args.host_limit:
            t = time.perf_counter()
            ref = brp.running_median(x, w)
            line += f", host {1e3 * (time.perf_counter() - t):.1f} ms, exact={np.array_equal(out, ref)}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
