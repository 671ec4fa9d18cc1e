"""Kernel-level operations of the MI355X pipeline.

`fft_path(nsamples)` says how the device transforms a given length: the
three-pass packed real FFT (csrc/hip/fft_passes.hip) when N/2 factors over the
compiled lengths, else a chirp-z transform over the smallest factorable
convolution length (csrc/hip/bluestein.hip) -- the lengths any padding -P of
the reference produces (demod_binary.c:226-244, 782).

`DeviceSearch` holds one work unit in HBM and runs template batches through
the native engine. `candidates()` takes any number of templates: it cuts them
into engine batches and keeps up to `max_in_flight` batches submitted (the next
batch is launched while the previous one runs, as the C++ search workers do),
returning the per-template candidate lists in template order. Nothing here
falls back to a host implementation: without a HIP device the engine raises.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass

import numpy as np

from .. import native

N_LEVELS = 5  # harmonic levels 1, 2, 4, 8, 16


@dataclass(frozen=True)
class FFTPath:
    kind: str        # "three-pass" or "chirp-z"
    nsamples: int    # real transform length N
    dft_len: int     # complex DFT length: N/2 (packed real transform) or N (odd N, chirp-z)
    conv_len: int    # chirp-z convolution length L (== dft_len for the three-pass path)
    factors: tuple   # (L1, L2, L3) of the three-pass transform that runs

    @property
    def work_ratio(self) -> float:
        """Device transform work relative to the three-pass path of this N
        (two length-L transforms per template on the chirp-z path)."""
        return 1.0 if self.kind == "three-pass" else 2.0 * self.conv_len / (self.nsamples / 2)


def fft_path(nsamples: int) -> FFTPath:
    brp = native()
    n = int(nsamples)
    if n % 2 == 0:
        f = brp.fft_plan(n // 2)
        if f is not None:
            return FFTPath("three-pass", n, n // 2, n // 2, tuple(f))
    mb = n if n % 2 else n // 2
    p = brp.bluestein_plan(mb)
    if p is None:
        raise ValueError(f"no device FFT plan for N = {n}")
    return FFTPath("chirp-z", n, mb, int(p[0]), tuple(p[1:]))


class DeviceSearch:
    """Per-work-unit device state: series in HBM, FFT plan, batched template kernels."""

    def __init__(self, geometry: dict, series: np.ndarray, device: int = 0, batch: int = 4, mu0: float | None = None):
        if not 1 <= batch <= 64:
            raise ValueError("batch must be in [1, 64] (candidate key packing)")
        s = np.ascontiguousarray(series, dtype=np.float32)
        if s.size < geometry["n_unpadded"]:
            raise ValueError(f"series has {s.size} samples, the geometry needs {geometry['n_unpadded']}")
        self.brp = native()
        self.geometry = geometry
        self.batch = batch
        self.path = fft_path(geometry["nsamples"])
        self.engine = self.brp.HipEngine()
        self.engine.init(device, batch)  # raises if no HIP device
        self.engine.setup(geometry, s, float(np.mean(s)) if mu0 is None else float(mu0))

    def whiten(self, options: dict, zaps, series: np.ndarray) -> np.ndarray:
        """Whitening + RFI zapping on the device; returns the whitened series."""
        return self.engine.whiten(options, zaps, np.ascontiguousarray(series, dtype=np.float32))

    def power_spectrum(self, P: float, tau: float, psi0: float):
        """Normalised power spectrum (fft_size bins) of one resampled template and its n_steps."""
        return self.engine.power_spectrum(float(P), float(tau), float(psi0))

    def candidates(self, P, tau, psi0, thresholds):
        """Above-threshold (bins, powers) per harmonic level for every template,
        in template order, with up to max_in_flight() batches on the device."""
        P = np.asarray(P, np.float32).ravel()
        tau = np.asarray(tau, np.float32).ravel()
        psi0 = np.asarray(psi0, np.float32).ravel()
        if not P.size == tau.size == psi0.size:
            raise ValueError("P, tau and psi0 must have one entry per template")
        thr = [float(t) for t in thresholds]
        if len(thr) != N_LEVELS:
            raise ValueError("one threshold per harmonic level (5)")
        depth = max(1, int(self.engine.max_in_flight()))
        out: list = []
        pending: deque = deque()
        for lo in range(0, P.size, self.batch):
            hi = min(P.size, lo + self.batch)
            if len(pending) == depth:
                out.extend(self.engine.complete())
                pending.popleft()
            self.engine.submit(P[lo:hi], tau[lo:hi], psi0[lo:hi], thr)
            pending.append(hi - lo)
        while pending:
            out.extend(self.engine.complete())
            pending.popleft()
        return out

    def fft_plan(self):
        """(M, L1, L2, L3) of the transform the engine runs (M = L on the chirp-z path)."""
        return self.engine.plan()

    def stats(self) -> dict:
        return self.engine.stats()
