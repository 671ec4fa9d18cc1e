"""Utilities: file formats, synthetic data, statistics."""
from . import synth  # noqa: F401
