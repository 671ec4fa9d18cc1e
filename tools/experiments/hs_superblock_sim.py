"""Coarse first-level rejection for the pruned harmonic sum (round-5 review
item): one bound per super-block of G 16-index blocks, each harmonic's maximum
read with one load of <= 4 entries from a pyramid level of cells wide enough
for the super-block's reach (2^w-bin cells, w per harmonic), before the
per-block bounds of hs_pruned_kernel. Host model on benchmark-template
spectra (CPU golden model, whitened WU, chi^2 thresholds at -A 0.08); prints
the flagged super-block fraction and the bound loads per 16-index block
(16 today: one load per harmonic per block).

usage: python tools/experiments/hs_superblock_sim.py   (caches spectra in /tmp/hsim)"""
import json, sys
import numpy as np
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
Path("/tmp/hsim").mkdir(exist_ok=True)
import hs_bound_sim as S
HARM=S.HARM; LEVEL_END=S.LEVEL_END
def run(k):
    ps, g = S.spectrum(k, f"/tmp/hsim/ps{k}.f32")
    w2, fhi = g["window_2"], g["fundamental_idx_hi"]
    hhi = min(g["harmonic_idx_hi"], g["fft_size"])
    ps = ps[:hhi].astype(np.float32)
    thr = np.array((18.139, 21.241, 26.269, 34.648, 48.958), np.float32)
    padded = np.concatenate([ps, np.zeros(4096, np.float32)])
    i_start = ((w2 - 8) // 16) * 16 + 8
    nblk = (hhi - i_start + 15) // 16
    cache = {}
    def cells(w):
        if w not in cache:
            n = (len(padded) + w - 1) // w
            c = np.zeros(n * w, np.float32); c[:len(padded)] = padded
            cache[w] = c.reshape(n, w).max(axis=1)
        return cache[w]
    def rmax(l, lo_i, hi_i, w):
        lo = (l * np.maximum(lo_i, 0) + 8) >> 4; hi = (l * np.maximum(hi_i, 0) + 8) >> 4
        sh = w.bit_length() - 1
        src = cells(w); a, b = lo >> sh, hi >> sh
        m = src[np.minimum(a, len(src)-1)]
        D = int((b - a).max())
        for d in range(1, D + 1):
            m = np.maximum(m, src[np.minimum(np.minimum(a + d, b), len(src)-1)])
        return m, D
    out = {}
    for G in (1, 2, 4, 8):
        nsb = (nblk + G - 1) // G
        ib = i_start + 16 * G * np.arange(nsb, dtype=np.int64)
        maxD = 0
        u = []
        for h in range(5):
            span = 16 * G if h == 4 else 16 * G + 4
            parts = []
            for l in HARM[:LEVEL_END[h]]:
                nb = (l * (span - 1) + 15) // 16 + 1
                w = 1
                while (nb + w - 1) // w + 1 > 4: w *= 2
                if G == 1: w = 1 if l < 4 else 8
                m, D = rmax(l, ib, ib + span - 1, w); maxD = max(maxD, D)
                parts.append(m)
            s = parts[0]
            if h >= 1: s = s + parts[1]
            if h >= 2: s = s + (parts[2] + parts[3])
            if h >= 3: s = s + (((parts[4] + parts[5]) + parts[6]) + parts[7])
            if h >= 4:
                t = parts[8]
                for p in parts[9:]: t = t + p
                s = s + t
            u.append(s)
        f = np.zeros(nsb, bool)
        for h in range(5):
            off = (1 << (h - 1)) if h else 0
            j_lo, j_hi = (ib + off) >> h, (ib + 16 * G - 1 + off) >> h
            f |= (j_hi >= w2) & (j_lo < fhi) & ~(u[h] <= thr[h])
        out[G] = dict(frac=round(float(f.mean()), 5), maxD=maxD, loads_per_block=round((16 + f.mean() * G * 16) / G, 3) if G > 1 else 16)
    return out
for k in (0, 1000, 3000):
    print(k, json.dumps(run(k)), flush=True)
