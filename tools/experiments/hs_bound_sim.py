"""Flagged-block fractions of the pruned harmonic sum's bound filter under
different bound constructions, on one benchmark-template spectrum computed on
the CPU (whitened reference WU, -P 3 -f 400 -A 0.08 -W). Host-only model of
csrc/hip/harmonic_sum.hip's hs_pruned_kernel; prints JSON lines.

usage: python tools/experiments/hs_bound_sim.py [template] [ps.f32 cache]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import boinc_app_eah_brp_amd as pkg  # noqa: E402

D = ROOT / "data" / "testwu"
HARM = [16, 8, 12, 4, 14, 10, 6, 2, 15, 13, 11, 9, 7, 5, 3, 1]
LEVEL_END = [1, 2, 4, 8, 16]  # harmonics summed up to level h: HARM[:LEVEL_END[h]]


def spectrum(k, cache):
    brp = pkg.native()
    brp.set_log_level(2)
    hdr, series, _ = brp.read_work_unit(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"))
    opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
    g = brp.derive_geometry(hdr, opt)
    if cache and Path(cache).exists():
        return np.fromfile(cache, dtype=np.float32), g
    zaps = brp.read_zaplist(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"))
    w = brp.cpu_whiten(series, g, opt, zaps)
    P, tau, psi = brp.read_template_bank(str(D / "stochastic_full.bank"))
    x, _, _ = brp.cpu_resample(w, g, float(np.float32(P[k])), float(np.float32(tau[k])), float(np.float32(psi[k])))
    ps = brp.cpu_power_spectrum(x, g["fft_size"])
    ps = np.asarray(ps, dtype=np.float32)
    if cache:
        ps.tofile(cache)
    return ps, g


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    ps, g = spectrum(k, sys.argv[2] if len(sys.argv) > 2 else None)
    w2, fhi = g["window_2"], g["fundamental_idx_hi"]
    hhi = min(g["harmonic_idx_hi"], g["fft_size"])
    ps = ps[:hhi].astype(np.float32)
    i_start = ((w2 - 8) // 16) * 16 + 8
    nblk = (hhi - i_start + 15) // 16
    ib = i_start + 16 * np.arange(nblk, dtype=np.int64)
    thr = np.array([float(t) for t in (sys.argv[3:8] if len(sys.argv) > 7 else
                                       (18.139, 21.241, 26.269, 34.648, 48.958))], dtype=np.float32)
    padded = np.concatenate([ps, np.zeros(64, np.float32)])

    def cells(width):
        n = (len(padded) + width - 1) // width
        c = np.zeros(n * width, np.float32)
        c[:len(padded)] = padded
        return c.reshape(n, width).max(axis=1)

    cell_cache = {w: cells(w) for w in (2, 4, 8, 16)}

    def f16_up(x):
        """x rounded up to the next fp16 value (the packed-fp16 bound phase's
        staging; an upper bound stays an upper bound)"""
        h = x.astype(np.float16)
        lo = h.astype(np.float32) < x
        h[lo] = np.nextafter(h[lo], np.float16(np.inf))
        return h.astype(np.float32)

    # fp16 bound phase: cells rounded up to fp16, and the <= 15 fp16 additions of
    # a level-4 sum (round-to-nearest, 2^-11 each) covered by a relative margin
    F16_MARGIN = np.float32(1.0 + 16 * 2.0 ** -11)
    cell_cache.update({-w: f16_up(cell_cache[w]) for w in (8, 16)})

    def rmax(l, lo_i, hi_i, width):
        """max over the bins harmonic l reaches for indices [lo_i, hi_i] (inclusive)"""
        lo = (l * np.maximum(lo_i, 0) + 8) >> 4
        hi = (l * np.maximum(hi_i, 0) + 8) >> 4
        if width == 1:
            src, a, b = padded, lo, hi
        elif width == -1:
            src, a, b = f16_up(padded), lo, hi
        else:
            sh = abs(width).bit_length() - 1
            src, a, b = cell_cache[width], lo >> sh, hi >> sh
        m = src[np.minimum(a, len(src) - 1)]
        for d in range(1, int((b - a).max()) + 1):
            m = np.maximum(m, src[np.minimum(np.minimum(a + d, b), len(src) - 1)])
        return m

    def bounds(spans, width_of):
        u = []
        for h in range(5):
            lo_i, hi_i = ib + spans[h][0], ib + spans[h][1] - 1
            s = None
            # reference order: 16, 8, then pairs / quads / octets summed first
            parts = [rmax(l, lo_i, hi_i, width_of(l)) for l in HARM[:LEVEL_END[h]]]
            s = parts[0]
            if h >= 1:
                s = s + parts[1]
            if h >= 2:
                s = s + (parts[2] + parts[3])
            if h >= 3:
                s = s + (((parts[4] + parts[5]) + parts[6]) + parts[7])
            if h >= 4:
                t = parts[8]
                for p in parts[9:]:
                    t = t + p
                s = s + t
            u.append(s)
        return u

    def flagged(u, margin=np.float32(1.0)):
        u = [x * margin for x in u]
        f = np.zeros(nblk, bool)
        per = []
        for h in range(5):
            off = (1 << (h - 1)) if h else 0
            j_lo, j_hi = (ib + off) >> h, (ib + 15 + off) >> h
            fh = (j_hi >= w2) & (j_lo < fhi) & ~(u[h] <= thr[h])
            per.append(float(fh.mean()))
            f |= fh
        waves = f[: nblk // 64 * 64].reshape(-1, 64)
        iters = np.ceil(waves.sum(axis=1) / 3.0)
        return dict(blocks=float(f.mean()), per_level=[round(p, 5) for p in per],
                    waves_any=float((waves.sum(axis=1) > 0).mean()), iters_per_wave=float(iters.mean()))

    span20 = [(0, 20)] * 5
    tight = [(0, 16), (1, 17), (2, 18), (4, 20), (0, 16)]
    cur = lambda l: 1 if l < 4 else 8  # noqa: E731
    l4only = [(0, 20)] * 4 + [(0, 16)]
    variants = {
        "round-2 first version (span 20, bins for l<4, 8-bin cells)": (span20, cur),
        "default: level 4 over its 16 indices, levels 0-3 span 20, 8-bin cells": (l4only, cur),
        "level 4 over its 16 indices, levels 0-3 span 20, 4-bin cells (BRP_HS_CELL=4)":
            (l4only, lambda l: 1 if l < 4 else 4),
        "per-level spans, 8-bin cells": (tight, cur),
        "per-level spans, 4-bin cells": (tight, lambda l: 1 if l < 4 else 4),
        "per-level spans, bins for l<8, 8-bin cells": (tight, lambda l: 1 if l < 8 else 8),
        "per-level spans, 4-bin l<8, 8-bin": (tight, lambda l: 1 if l < 4 else (4 if l < 8 else 8)),
        "default, 16-bin cells": (l4only, lambda l: 1 if l < 4 else 16),
        "default, fp16 bound phase (cells/bins rounded up to fp16, +16 ulp margin)":
            (l4only, lambda l: -1 if l < 4 else -8),
        "default, fp16 bound phase with 16-bin cells": (l4only, lambda l: -1 if l < 4 else -16),
        "per-level spans, exact bins": (tight, lambda l: 1),
        "span 20, exact bins": (span20, lambda l: 1),
    }
    for name, (sp, wf) in variants.items():
        margin = F16_MARGIN if "fp16" in name else np.float32(1.0)
        print(json.dumps(dict(variant=name, template=k, thr=thr.tolist(), **flagged(bounds(sp, wf), margin))),
              flush=True)


if __name__ == "__main__":
    main()
