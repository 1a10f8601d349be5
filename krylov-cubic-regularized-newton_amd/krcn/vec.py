"""Handle-free device vector kernels (krcn_vctx): the Lanczos recurrence over an
external operator and the dense helpers of the host loops.

`optimizer.cubic.Lanczos(A, v, m)` with a plain callable A (the reference's
`lambda v: loss.hess_vec_prod(x, v)`, cubic.py:273) cannot use the fused
device recurrence of krcn_lanczos, which owns the HVP; it calls A once per
step instead and runs every vector operation of cubic.py:85-109 here, on the
device, through krcn_lz_ext_step / krcn_vec_div / krcn_vec_dot.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib
from ._lib import call

_DTYPES = {torch.float64: _lib.KRCN_F64, torch.float32: _lib.KRCN_F32}


def _p(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


class VecContext:
    """Reduction scratch on one device (krcn_vctx_create)."""

    _cache = {}
    _lock = threading.Lock()

    def __init__(self, device):
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._h = ctypes.c_void_p()
        call("krcn_vctx_create", self.device.index, ctypes.byref(self._h))

    @classmethod
    def for_device(cls, device):
        """The context of (device, torch's current stream there): a context's
        reduction scratch is reused by every call, so two streams (or the host
        threads of virtual ranks, krcn.dist.VirtualShards) each get their own."""
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        key = (idx, torch.cuda.current_stream(idx).cuda_stream)
        ctx = cls._cache.get(key)
        if ctx is None:
            with cls._lock:
                ctx = cls._cache.get(key)
                if ctx is None:
                    ctx = cls._cache[key] = cls(torch.device("cuda", idx))
        return ctx

    def close(self):
        if self._h.value:
            _lib.load().krcn_vctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _check(*ts):
        t0 = ts[0]
        for t in ts:
            if t is None:
                continue
            if t.dtype != t0.dtype or t.dim() != 1 or not t.is_contiguous() or t.numel() != t0.numel():
                raise ValueError("vectors must be contiguous 1-D tensors of one dtype and length")
        if t0.dtype not in _DTYPES:
            raise TypeError(f"dtype must be float64 or float32, got {t0.dtype}")
        return _DTYPES[t0.dtype], t0.numel()

    def lz_step(self, y, v, v_pre, beta, z):
        """z = (y - beta v_pre) - alpha v with alpha = v.(y - beta v_pre); returns (alpha, ||z||)."""
        code, n = self._check(y, v, v_pre, z)
        ab = np.zeros(2)
        call("krcn_lz_ext_step", self._h, code, n, _p(y), _p(v), _p(v_pre), float(beta), _p(z),
             ab.ctypes.data_as(_lib._dp), self._stream())
        return float(ab[0]), float(ab[1])

    def dot(self, a, b) -> float:
        code, n = self._check(a, b)
        out = ctypes.c_double()
        call("krcn_vec_dot", self._h, code, n, _p(a), _p(b), ctypes.byref(out), self._stream())
        return float(out.value)

    def div(self, a, div, out=None):
        code, n = self._check(a, out)
        out = torch.empty_like(a) if out is None else out
        call("krcn_vec_div", self._h, code, n, _p(a), float(div), _p(out), self._stream())
        return out

    def axpy(self, alpha, x, y, out=None):
        """y + alpha x."""
        code, n = self._check(x, y, out)
        out = torch.empty_like(y) if out is None else out
        call("krcn_vec_axpy", self._h, code, n, float(alpha), _p(x), _p(y), _p(out), self._stream())
        return out
