"""MI355X-native Einstein@Home binary radio pulsar (BRP) search.

A from-scratch re-design of the capabilities of boinc-app-eah-brp for AMD
Instinct MI355X (gfx950): the per-template pipeline (time-domain resampling,
3*2^n-point real FFT + power spectrum, 16-harmonic summing, candidate
selection) runs as hand-written HIP kernels, templates stream through three
pipelines (HIP streams) per GPU with two batches in flight each (HIP graph
replay optional, BRP_GRAPH=1), and template banks are sharded over GPUs with
RCCL all-gathers of the candidate tables.

Layout:
  models/    search pipelines (GPU search, CPU golden model, numpy oracle)
  ops/       device operations (power spectrum, harmonic sums, whitening)
  parallel/  multi-GPU sharding over torch.distributed (RCCL / gloo)
  utils/     file formats, synthetic data, statistics
The native code lives in csrc/ and is built in-tree by `_build.py`.
"""
from __future__ import annotations

import importlib
import os
import sys

__version__ = "0.1.0"

_native = None


def native():
    """Return the compiled extension module, building it on first use if needed."""
    global _native
    if _native is not None:
        return _native
    # torch (when present) must load its HIP runtime first so both share one copy
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional for CPU-only use
            pass
    # BRP_CHECKED=1: the device-side debug build (csrc/hip/checked.hpp)
    checked = os.environ.get("BRP_CHECKED", "0") not in ("", "0")
    name = "._brp_checked" if checked else "._brp"
    try:
        _native = importlib.import_module(name, __name__)
    except ImportError:
        if os.environ.get("BRP_NO_AUTOBUILD"):
            raise
        from . import _build

        if checked:
            _build.build_checked(verbose=False)
        else:
            _build.build(verbose=False)
        _native = importlib.import_module(name, __name__)
    return _native


def __getattr__(name):  # lazy access: boinc_app_eah_brp_amd.models etc.
    if name in ("models", "ops", "parallel", "utils"):
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
