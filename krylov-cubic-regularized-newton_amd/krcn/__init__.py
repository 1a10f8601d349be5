"""krcn — MI355X-native Krylov cubic-regularized-Newton hot path.

The native library (lib/libkrcn.so, sources in csrc/, ABI in include/krcn.h)
holds the HIP kernels; this package is its Python face: the device matrix
handle, the deterministic synthetic problem generator, and multi-GPU sharding.
"""
from . import synth  # noqa: F401
from ._lib import (KRCN_FORMAT_AUTO, KRCN_FORMAT_SORTED, KRCN_FORMAT_WAVE,  # noqa: F401
                   KRCN_FORMAT_JAG, KRCN_FORMAT_WINDOW, KrcnError, load)
from .device import DeviceCSR  # noqa: F401

__all__ = ["DeviceCSR", "KrcnError", "load", "synth"]
