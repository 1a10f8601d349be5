"""Device-resident sparse design matrix: the Python face of a krcn_csr handle.

`DeviceCSR` uploads a scipy CSR matrix (the reference's LogisticRegression.A,
optimizer/loss.py:188) to HBM as torch tensors, asks libkrcn to build the
explicit, row-order-stable transpose (the reference multiplies by the zero-copy
CSC view A.T, loss.py:227,302), and exposes every C-ABI entry point as a method
taking torch device tensors.  All launches go to torch's current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import call

_DTYPES = {torch.float64: _lib.KRCN_F64, torch.float32: _lib.KRCN_F32}


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class DeviceCSR:
    """X (n x d) in CSR on one GPU, plus X^T in CSR, behind libkrcn.

    shard_mode / n_global describe how this block relates to the global matrix
    (include/krcn.h, KRCN_SHARD_*).  Vectors passed to the methods have the
    block's local lengths: n-vectors of length `n`, d-vectors of length `d`.
    """

    def __init__(self, A, device=None, dtype=torch.float64, n_global=None,
                 shard_mode=_lib.KRCN_SHARD_NONE, lanes=(0, 0), slicing=0, fmt=0, pass_formats=None):
        if not torch.cuda.is_available():
            raise RuntimeError("krcn.DeviceCSR needs a HIP device (no CPU fallback exists)")
        if dtype not in _DTYPES:
            raise TypeError(f"dtype must be torch.float64 or torch.float32, got {dtype}")
        A = sp.csr_matrix(A)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        self.n, self.d = (int(s) for s in A.shape)
        self.nnz = int(A.nnz)
        self.n_global = int(n_global) if n_global is not None else self.n
        self.shard_mode = shard_mode
        self.indptr = torch.from_numpy(np.ascontiguousarray(A.indptr, dtype=np.int32)).to(self.device)
        self.indices = torch.from_numpy(np.ascontiguousarray(A.indices, dtype=np.int32)).to(self.device)
        np_dt = np.float64 if dtype == torch.float64 else np.float32
        self.data = torch.from_numpy(np.ascontiguousarray(A.data, dtype=np_dt)).to(self.device)
        self._h = ctypes.c_void_p()
        self._comm = None
        self._fn_lanczos = _lib.load().krcn_lanczos
        self._lz_bufs = None
        self._reorth_m = 0       # CGS2 workspace reserved for Lanczos m <= this
        _lib.load()
        # the uploads above ran on the current stream; the library builds on its own
        torch.cuda.current_stream(self.device).synchronize()
        call("krcn_csr_create", self.device.index, self.n, self.d, self.nnz, _ptr(self.indptr),
             _ptr(self.indices), _ptr(self.data), _DTYPES[dtype], self.n_global, shard_mode,
             ctypes.byref(self._h))
        self.set_lanes(*lanes)
        self.set_slicing(slicing)
        self.set_format(fmt)
        if pass_formats is not None:
            for k, f in enumerate(pass_formats):
                self.set_pass_format(k + 1, f)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().krcn_csr_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def owned_bytes(self) -> int:
        b = ctypes.c_int64()
        call("krcn_csr_owned_bytes", self._h, ctypes.byref(b))
        return int(b.value)

    def set_lanes(self, lanes_x=0, lanes_xt=0):
        """Row-group width for X / X^T kernels: 0 auto, 1 sequential (scipy order), 2..64."""
        call("krcn_csr_set_lanes", self._h, int(lanes_x), int(lanes_xt))
        self._replan()

    def set_slicing(self, slicing=0):
        """0 auto, 1 off, or a forced slice count (multiple of 8) for both passes."""
        call("krcn_csr_set_slicing", self._h, int(slicing))
        self._replan()

    def set_format(self, fmt=0):
        """Tile format: 0 auto, 1 wave tiles (CSR order), 2 sorted block tiles, 3 LDS windows, 4 jagged."""
        call("krcn_csr_set_format", self._h, int(fmt))
        self._replan()

    def set_pass_format(self, pass_, fmt):
        """Tile format of one pass (1: X, 2: X^T), overriding set_format for it; -1 restores it."""
        call("krcn_csr_set_pass_format", self._h, int(pass_), int(fmt))
        self._replan()

    def _multi_rank(self):
        return self._comm is not None and getattr(self._comm, "world", 1) > 1

    def _replan(self):
        # a handle of a multi-rank communicator builds plans only in explicit
        # calls, never inside a compute call its peers wait on (include/krcn.h)
        if self._multi_rank():
            self.reserve(1)

    def reserve(self, m_max, reorth=False):
        """Build the pass plans and reserve krcn_lanczos's workspace for m <= m_max
        (krcn_csr_reserve): later lanczos calls up to m_max allocate nothing."""
        call("krcn_csr_reserve", self._h, int(m_max), int(bool(reorth)))
        if reorth:
            self._reorth_m = max(self._reorth_m, int(m_max))

    def set_graph(self, on=True):
        """hipGraph replay of repeated lanczos() calls (krcn_csr_set_graph; off by default)."""
        call("krcn_csr_set_graph", self._h, int(bool(on)))

    def set_placement_trials(self, trials=-1):
        """Placement probe at plan builds (krcn_csr_set_placement_trials): -1 auto, 0 off, 1..8."""
        call("krcn_csr_set_placement_trials", self._h, int(trials))
        self._replan()

    def placement_info(self):
        """The placement probe of the last plan build ({'probed', 'kept', 'hot_mb', 'policy', 'us': [per
        placement, probe HVP]}) and the search over the first Lanczos calls ({'lanczos': {'timed', 'kept',
        'm', 'ms': [per placement, one call each]}})."""
        buf = (ctypes.c_double * 24)()
        call("krcn_csr_placement_info", self._h, buf)
        k, kl = int(buf[0]), int(buf[12])
        return {"probed": k, "kept": int(buf[1]), "hot_mb": round(buf[2], 1), "policy": int(buf[3]),
                "us": [round(buf[4 + i], 2) for i in range(k)],
                "lanczos": {"timed": kl, "kept": int(buf[13]), "m": int(buf[14]),
                            "ms": [round(buf[16 + i], 4) for i in range(kl)]}}

    def plan_info(self):
        """{'pass1': (slices, lanes, tiles, grid), 'pass2': (...)}; slices < 0 marks sorted tiles."""
        buf = (ctypes.c_int * 8)()
        call("krcn_csr_plan_info", self._h, buf)
        return {"pass1": tuple(buf[0:4]), "pass2": tuple(buf[4:8])}

    _FORMAT_NAMES = {1: "wave", 2: "sorted", 3: "window-slices", 4: "window-accum", 5: "jagged"}

    def plan_format(self):
        """{'pass1': name, 'pass2': name}: wave, sorted, window-slices or window-accum."""
        buf = (ctypes.c_int * 2)()
        call("krcn_csr_plan_format", self._h, buf)
        return {"pass1": self._FORMAT_NAMES[buf[0]], "pass2": self._FORMAT_NAMES[buf[1]]}

    def attach_comm(self, comm):
        call("krcn_csr_attach_comm", self._h, comm.handle if comm is not None else None)
        self._comm = comm

    def transpose_arrays(self):
        """(colptr, rowidx, vals) of the device-built X^T, as device tensors."""
        colptr = torch.empty(self.d + 1, dtype=torch.int32, device=self.device)
        rowidx = torch.empty(self.nnz, dtype=torch.int32, device=self.device)
        vals = torch.empty(self.nnz, dtype=self.dtype, device=self.device)
        call("krcn_csr_get_transpose", self._h, _ptr(colptr), _ptr(rowidx), _ptr(vals),
             _stream(self.device))
        return colptr, rowidx, vals

    # -- helpers -----------------------------------------------------------
    def _check(self, t, length, name):
        if t is None:
            raise ValueError(f"{name} is required")
        if not isinstance(t, torch.Tensor) or t.device != self.device:
            raise TypeError(f"{name} must be a torch tensor on {self.device}")
        if t.dtype != self.dtype:
            raise TypeError(f"{name} must have dtype {self.dtype}, got {t.dtype}")
        if not t.is_contiguous() or t.dim() != 1 or t.numel() != length:
            raise ValueError(f"{name} must be a contiguous 1-D tensor of length {length}, "
                             f"got shape {tuple(t.shape)}")
        return t

    def empty_n(self):
        return torch.empty(self.n, dtype=self.dtype, device=self.device)

    def empty_d(self):
        return torch.empty(self.d, dtype=self.dtype, device=self.device)

    # -- objective pieces --------------------------------------------------
    def matvec(self, x, out=None):
        """Ax = X x (loss.py:270)."""
        self._check(x, self.d, "x")
        out = self.empty_n() if out is None else self._check(out, self.n, "out")
        call("krcn_matvec", self._h, _ptr(x), _ptr(out), _stream(self.device))
        return out

    def rmatvec(self, u, out=None):
        """y = X^T u / n_global (loss.py:227,302)."""
        self._check(u, self.n, "u")
        out = self.empty_d() if out is None else self._check(out, self.d, "out")
        call("krcn_rmatvec", self._h, _ptr(u), _ptr(out), _stream(self.device))
        return out

    def weights(self, Ax, out=None):
        """w = s(1-s), s = expit(Ax) (loss.py:296-297)."""
        self._check(Ax, self.n, "Ax")
        out = self.empty_n() if out is None else self._check(out, self.n, "out")
        call("krcn_weights", self._h, _ptr(Ax), _ptr(out), _stream(self.device))
        return out

    def hvp(self, w, v, out=None, l2=0.0):
        """y = X^T (w * X v) / n + l2 v (loss.py:289-302)."""
        self._check(w, self.n, "w")
        self._check(v, self.d, "v")
        out = self.empty_d() if out is None else self._check(out, self.d, "out")
        call("krcn_hvp", self._h, _ptr(w), _ptr(v), _ptr(out), float(l2), _stream(self.device))
        return out

    def gradient(self, Ax, b, x=None, l2=0.0, out=None):
        """grad = X^T (expit(Ax) - b) / n (+ l2 x) (loss.py:223-232)."""
        self._check(Ax, self.n, "Ax")
        self._check(b, self.n, "b")
        if l2 != 0.0:
            self._check(x, self.d, "x")
        out = self.empty_d() if out is None else self._check(out, self.d, "out")
        call("krcn_gradient", self._h, _ptr(Ax), _ptr(b), _ptr(x), float(l2), _ptr(out),
             _stream(self.device))
        return out

    def loss_mean(self, Ax, b) -> float:
        """mean((1-b) Ax - logsig(Ax)) (loss.py:215-220 without the l2 term)."""
        self._check(Ax, self.n, "Ax")
        self._check(b, self.n, "b")
        out = ctypes.c_double()
        call("krcn_loss_mean", self._h, _ptr(Ax), _ptr(b), ctypes.byref(out), _stream(self.device))
        return float(out.value)

    def loss_values(self, xs, b):
        """[loss_mean(matvec(x), b) for x in xs] in one submission and one sync
        (krcn_loss_values): each value bitwise the per-iterate one."""
        self._check(b, self.n, "b")
        for i, x in enumerate(xs):
            self._check(x, self.d, f"xs[{i}]")
        k = len(xs)
        out = np.zeros(max(k, 1), dtype=np.float64)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[x.data_ptr() for x in xs])
        call("krcn_loss_values", self._h, k, ptrs, _ptr(b), out.ctypes.data_as(_lib._dp),
             _stream(self.device))
        return [float(v) for v in out[:k]]

    # -- Lanczos -----------------------------------------------------------
    def lanczos(self, w, g, m, reorth=False, tol=1e-6, l2=0.0, V=None):
        """Three-term Lanczos on v -> hvp(w, v) from g (cubic.py:77-111).

        Returns (V, alphas, betas, info): V a device tensor of m rows x d (row j
        is the reference's column V[:, j]; rows >= info.m_eff are not part of
        the basis), alphas (m_eff,) and betas (m_eff-1,) numpy float64 arrays.
        """
        m = int(m)
        if m < 1:
            raise ValueError("m must be >= 1")
        self._check(w, self.n, "w")
        self._check(g, self.d, "g")
        if V is None:
            V = torch.empty((m, self.d), dtype=self.dtype, device=self.device)
        elif (V.dtype != self.dtype or V.device != self.device or not V.is_contiguous()
              or tuple(V.shape) != (m, self.d)):
            raise ValueError(f"V must be a contiguous ({m}, {self.d}) {self.dtype} tensor on {self.device}")
        if reorth and m > self._reorth_m:
            self.reserve(m, reorth=True)   # before the recurrence, not inside it
        # host result buffers reused across calls (w8a's m = 10 calls are
        # ~165 us each: the wrapper's own allocations showed up); the
        # returned arrays are copies
        if self._lz_bufs is None or self._lz_bufs[0].size < m:
            cap = max(m, 64)
            al_b, be_b = np.zeros(cap, dtype=np.float64), np.zeros(cap, dtype=np.float64)
            self._lz_bufs = (al_b, be_b, al_b.ctypes.data_as(_lib._dp), be_b.ctypes.data_as(_lib._dp))
        al_b, be_b, al_p, be_p = self._lz_bufs
        info = _lib.LanczosInfo()
        st = self._fn_lanczos(self._h, _ptr(w), _ptr(g), m, int(bool(reorth)), float(tol), float(l2),
                              _ptr(V), al_p, be_p, ctypes.byref(info), _stream(self.device))
        if st != _lib.KRCN_OK:
            msg = _lib.load().krcn_last_error_string()
            raise _lib.KrcnError(st, "krcn_lanczos", msg.decode() if msg else "")
        me = info.m_eff
        return V, al_b[:me].copy(), be_b[:max(me - 1, 0)].copy(), info

    def cg_solve(self, w, b, shift=0.0, rtol=1e-5, maxiter=None, out=None):
        """x ~= (H + shift I)^{-1} b, H = X^T diag(w) X / n, by device conjugate
        gradients with scipy.sparse.linalg.cg's loop and stopping rule (x0 = 0,
        stop when ||r|| < rtol ||b||, maxiter default 10 d).  Returns (x, info)."""
        self._check(w, self.n, "w")
        self._check(b, self.d, "b")
        out = self.empty_d() if out is None else self._check(out, self.d, "out")
        maxiter = 10 * self.d if maxiter is None else int(maxiter)
        info = _lib.CgInfo()
        call("krcn_cg_solve", self._h, _ptr(w), _ptr(b), float(shift), float(rtol), maxiter, _ptr(out),
             ctypes.byref(info), _stream(self.device))
        return out, info

    def basis_combine(self, V, s, x, out=None):
        """x + V^T s over the first len(s) basis rows (cubic.py:291)."""
        s = np.ascontiguousarray(s, dtype=np.float64)
        self._check(x, self.d, "x")
        if V.dim() != 2 or V.shape[1] != self.d or V.shape[0] < len(s):
            raise ValueError("V must be (>= len(s)) x d")
        out = self.empty_d() if out is None else self._check(out, self.d, "out")
        call("krcn_basis_combine", self._h, len(s), _ptr(V), s.ctypes.data_as(_lib._dp), _ptr(x),
             _ptr(out), _stream(self.device))
        return out

    # -- vector helpers ----------------------------------------------------
    def _space_len(self, space):
        return self.n if space == _lib.KRCN_SPACE_N else self.d

    def dot(self, a, b, space=_lib.KRCN_SPACE_D) -> float:
        ln = self._space_len(space)
        self._check(a, ln, "a")
        self._check(b, ln, "b")
        out = ctypes.c_double()
        call("krcn_dot", self._h, space, _ptr(a), _ptr(b), ctypes.byref(out), _stream(self.device))
        return float(out.value)

    def diff_norm(self, a, b=None, space=_lib.KRCN_SPACE_D) -> float:
        ln = self._space_len(space)
        self._check(a, ln, "a")
        if b is not None:
            self._check(b, ln, "b")
        out = ctypes.c_double()
        call("krcn_diff_norm", self._h, space, _ptr(a), _ptr(b), ctypes.byref(out),
             _stream(self.device))
        return float(out.value)

    # -- profiling ---------------------------------------------------------
    def prof_enable(self, on=True):
        call("krcn_prof_enable", self._h, int(bool(on)))

    def prof_read(self):
        """{'count', 'pass1_ms' (with its slice combine), 'pass2_ms', 'hvp_ms',
        'pass1_kernel_ms', 'combine_ms'} accumulated since enable/last read."""
        buf = (ctypes.c_double * 8)()
        call("krcn_prof_read", self._h, buf)
        return {"count": int(buf[0]), "pass1_ms": buf[1], "pass2_ms": buf[3], "hvp_ms": buf[5],
                "pass1_kernel_ms": buf[6], "combine_ms": buf[7]}
