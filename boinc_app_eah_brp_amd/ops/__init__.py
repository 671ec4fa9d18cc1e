"""Device operations of the MI355X pipeline.

Thin, explicit wrappers over the native HIP engine. They never fall back to a
host implementation: on a machine without a HIP device they raise.
"""
from __future__ import annotations

import numpy as np

from .. import native


class DeviceSearch:
    """Per-work-unit device state: series in HBM, FFT plan, batched template kernels."""

    def __init__(self, geometry: dict, series: np.ndarray, device: int = 0, batch: int = 4, mu0: float | None = None):
        self.brp = native()
        self.geometry = geometry
        self.engine = self.brp.HipEngine()
        self.engine.init(device, batch)  # raises if no HIP device
        s = np.ascontiguousarray(series, dtype=np.float32)
        self.engine.setup(geometry, s, float(np.mean(s)) if mu0 is None else float(mu0))

    def whiten(self, options: dict, zaps, series: np.ndarray) -> np.ndarray:
        """Whitening + RFI zapping on the device; returns the whitened series."""
        return self.engine.whiten(options, zaps, np.ascontiguousarray(series, dtype=np.float32))

    def power_spectrum(self, P: float, tau: float, psi0: float):
        """Normalised power spectrum (fft_size bins) of one resampled template and its n_steps."""
        return self.engine.power_spectrum(float(P), float(tau), float(psi0))

    def candidates(self, P, tau, psi0, thresholds):
        """Above-threshold bins per harmonic level for a batch of templates."""
        P = np.asarray(P, np.float32).ravel()
        tau = np.asarray(tau, np.float32).ravel()
        psi0 = np.asarray(psi0, np.float32).ravel()
        return self.engine.process(P, tau, psi0, [float(t) for t in thresholds])

    def fft_plan(self):
        return self.engine.plan()

    def stats(self) -> dict:
        return self.engine.stats()
