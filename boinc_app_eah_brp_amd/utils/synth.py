"""Synthetic work units, template banks and binary-pulsar injections.

There is no network access to Einstein@Home data; besides the one benchmark WU
shipped with the reference (data/testwu) all test and benchmark inputs are
generated here with the same on-disk formats (1168-byte header + 4-bit or 8-bit
payload, "%lg %lg %lg" bank lines).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from .. import native


@dataclass
class Injection:
    f0: float = 0.0        # spin frequency [Hz] (0: no signal)
    P_orb: float = 1000.0  # orbital period [s]
    tau: float = 0.0       # projected orbital radius [lt-s]
    psi0: float = 0.0      # initial orbital phase [rad]
    amplitude: float = 0.5  # pulse amplitude in units of the noise sigma
    duty: float = 0.1      # pulse duty cycle


def make_series(n: int, tsample_us: float, inj: Injection | None = None, seed: int = 0,
                mean: float = 7.5, sigma: float = 2.0) -> np.ndarray:
    """Float time series: white noise plus an optional binary pulsar."""
    rng = np.random.default_rng(seed)
    x = rng.normal(mean, sigma, n)
    if inj is not None and inj.f0 > 0:
        dt = tsample_us * 1e-6
        t = np.arange(n) * dt
        omega = 2 * math.pi / inj.P_orb
        # pulsar proper time of the detector sample (Roemer delay of a circular orbit)
        tp = t + inj.tau * np.sin(omega * t + inj.psi0) - inj.tau * math.sin(inj.psi0)
        phase = np.mod(inj.f0 * tp, 1.0)
        x += inj.amplitude * sigma * (phase < inj.duty) / inj.duty * 0.5
    return x


def quantize_4bit(x: np.ndarray) -> np.ndarray:
    """Pack samples (already in units of the 0..15 grid) as 4-bit pairs, high nibble first."""
    q = np.clip(np.rint(x), 0, 15).astype(np.uint8)
    if q.size % 2:
        q = np.append(q, 0)
    return (q[0::2] << 4) | q[1::2]


def quantize_8bit(x: np.ndarray, mean: float = 7.5) -> np.ndarray:
    q = np.clip(np.rint((x - mean) * 8.0), -128, 127).astype(np.int8)
    return q.view(np.uint8)


def write_wu(path: str | Path, x: np.ndarray, tsample_us: float = 65.476, four_bit: bool = True,
             scale: float = 1.0, gzip: bool = True, **hdr) -> Path:
    path = Path(path)
    payload = quantize_4bit(x) if four_bit else quantize_8bit(x)
    header = dict(tsample=tsample_us, tobs=x.size * tsample_us * 1e-6, nsamples=int(x.size), scale=scale,
                  DM=hdr.pop("DM", 100.0), RA=hdr.pop("RA", 55920.56), DEC=hdr.pop("DEC", 220748.1),
                  name=hdr.pop("name", "SYNTH"), originalfile=hdr.pop("originalfile", "synthetic"))
    header.update(hdr)
    native().write_work_unit(str(path), header, payload, gzip)
    return path


def write_bank(path: str | Path, P, tau, psi) -> Path:
    path = Path(path)
    with open(path, "w") as fh:
        for a, b, c in zip(P, tau, psi):
            fh.write(f"{a:.12f} {b:.12f} {c:.12f}\n")
    return path


def random_bank(n: int, seed: int = 1, P_range=(660.0, 2231.0), tau_max=0.335, include=None):
    """Random circular-orbit template bank like stochastic_full.bank
    (P_orb 660-2231 s, tau 0-0.335 s, Psi0 0-2pi); `include` prepends exact templates."""
    rng = np.random.default_rng(seed)
    P = rng.uniform(*P_range, n)
    tau = rng.uniform(0.0, tau_max, n)
    psi = rng.uniform(0.0, 2 * math.pi, n)
    P[0], tau[0], psi[0] = 1000.0, 0.0, 0.0  # the reference bank starts with the unmodulated template
    if include:
        extra = np.array(include, dtype=float).reshape(-1, 3)
        P = np.concatenate([extra[:, 0], P])
        tau = np.concatenate([extra[:, 1], tau])
        psi = np.concatenate([extra[:, 2], psi])
    return P, tau, psi


def write_zaplist(path: str | Path, ranges) -> Path:
    path = Path(path)
    with open(path, "w") as fh:
        for lo, hi in ranges:
            fh.write(f"{lo} {hi}\n")
    return path


def synthetic_case(workdir: str | Path, n: int = 1 << 16, n_templates: int = 16, inj: Injection | None = None,
                   seed: int = 0, tsample_us: float = 65.476) -> dict:
    """A complete small search setup (WU, bank, zaplist) in `workdir`."""
    workdir = Path(workdir)
    workdir.mkdir(parents=True, exist_ok=True)
    x = make_series(n, tsample_us, inj, seed)
    wu = write_wu(workdir / "synth.bin4", x, tsample_us)
    include = [(inj.P_orb, inj.tau, inj.psi0)] if inj is not None and inj.f0 > 0 else None
    P, tau, psi = random_bank(n_templates, seed + 1, include=include)
    bank = write_bank(workdir / "synth.bank", P, tau, psi)
    zap = write_zaplist(workdir / "synth.zap", [(59.9, 60.1), (119.9, 120.1)])
    return dict(wu=str(wu), bank=str(bank), zap=str(zap), P=P, tau=tau, psi=psi, series=x)
