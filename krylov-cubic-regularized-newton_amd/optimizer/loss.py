"""Logistic-regression oracle on the GPU (drop-in for optimizer/loss.py).

Same constructor and methods as the reference's `LogisticRegression`
(loss.py:179-302): value, gradient, hess_vec_prod, mat_vec_product, reset, n,
dim, f_opt, x_opt.  The design matrix lives in HBM behind a libkrcn handle
(krcn.DeviceCSR); every product with X or X^T is a hand-written gfx950 kernel.

Vectors: methods accept numpy arrays (returning numpy, as the reference does)
or torch tensors on the handle's device (returning device tensors — the
Krylov-CRN step keeps everything on the GPU this way).

Caching (loss.py:266-277, store_mat_vec_prod=True): Ax and the Hessian weights
s(1-s) are kept for the last x.  A device x hits the cache when it is the same
tensor object at the same version (the cache holds a reference, so its memory
cannot be recycled under it); a numpy x hits when it is array_equal to the
last numpy x, the reference's own test (loss.py:361-375).  The weights are
recomputed only when Ax changes — the reference recomputes them on every HVP
(loss.py:296-297) with identical results.

Out of scope: dense `hessian`, the SSCN `partial_*` methods, l1 /
prox regularizers and the smoothness estimates; they raise NotImplementedError.
"""
from __future__ import annotations

import copy
import warnings

import numpy as np
import torch

import krcn
from krcn import _lib
from krcn.labels import labels01 as _labels01


class Oracle:
    """Base objective (loss.py:29-113): l1/l2 coefficients and best-value tracking."""

    def __init__(self, l1=0, l2=0, l2_in_prox=False, regularizer=None, seed=42):
        if l1 < 0.0:
            raise ValueError(f"Invalid value for l1 regularization: {l1}")
        if l2 < 0.0:
            raise ValueError(f"Invalid value for l2 regularization: {l2}")
        if l2 == 0.0 and l2_in_prox:
            warnings.warn("The value of l2 is set to 0, so l2_in_prox is changed to False.")
            l2_in_prox = False
        self.l1 = l1
        self.l2 = 0 if l2_in_prox else l2
        self.l2_in_prox = l2_in_prox
        self.x_opt = None
        self.f_opt = np.inf
        self.regularizer = regularizer
        self.seed = seed
        if (l1 > 0 or l2_in_prox) or regularizer is not None:
            raise NotImplementedError(
                "l1 / prox regularizers are outside the device hot path (SURVEY.md §2)")
        self.rng = np.random.default_rng(seed)

    def set_seed(self, seed):
        self.seed = seed
        self.rng = np.random.default_rng(seed)

    def value(self, x):
        """Objective value with best-iterate tracking (loss.py:66-73)."""
        val = self._value(x)
        if val < self.f_opt:
            self.x_opt = x.clone() if isinstance(x, torch.Tensor) else copy.deepcopy(x)
            self.f_opt = val
        return val


class HessianOperator:
    """v -> hess_vec_prod(x, v) at a fixed x, on the device.

    The reference builds `lambda v: loss.hess_vec_prod(self.x, v)`
    (cubic.py:273) and hands it to Lanczos; passing this object instead lets
    `optimizer.cubic.Lanczos` run the fused device recurrence."""

    def __init__(self, loss, x):
        self.loss = loss
        self.x = x
        self.X = loss.device_matrix
        self.w = loss._weights_for(x)
        self.l2 = float(loss.l2)

    def __call__(self, v):
        return self.loss.hess_vec_prod(self.x, v)


class LogisticRegression(Oracle):
    """Logistic loss f(x) = mean((1-b) Ax - logsig(Ax)) (+ l2/2 ||x||^2) on the GPU.

    A: scipy sparse (converted to CSR) or dense n x d matrix; b: binary labels.
    device / dtype: where and in which precision the device copy of A lives
    (fp64 by default, as the reference computes).  shard: optional
    krcn.dist.ShardSpec for multi-GPU runs (krcn.dist.shard_problem builds it).
    """

    def __init__(self, A, b, store_mat_vec_prod=False, *args, device=None, dtype=torch.float64,
                 shard=None, lanes=(0, 0), **kwargs):
        super().__init__(*args, **kwargs)
        import scipy.sparse as sp
        self.A = A
        self.b = _labels01(b)
        self.store_mat_vec_prod = store_mat_vec_prod
        self.reuse = False
        self.shard = shard
        A_local = sp.csr_matrix(A) if shard is None else shard.A_local
        b_local = np.asarray(self.b, dtype=np.float64) if shard is None else shard.b_local(self.b)
        self.n, self.dim = A.shape
        mode = _lib.KRCN_SHARD_NONE if shard is None else shard.mode
        self.device_matrix = krcn.DeviceCSR(A_local, device=device, dtype=dtype,
                                            n_global=self.n, shard_mode=mode, lanes=lanes)
        if shard is not None and shard.comm is not None:
            self.device_matrix.attach_comm(shard.comm)
        self.device = self.device_matrix.device
        self.dtype = dtype
        self._b_dev = torch.from_numpy(b_local.astype(self._np_dtype())).to(self.device)
        self.x_last = 0.0
        self._mat_vec_prod = None
        self._cache_x = None        # device tensor whose Ax is cached
        self._cache_ver = None
        self._cache_np = None       # numpy copy for array_equal hits
        self._w = None

    # ------------------------------------------------------------ vectors
    def _np_dtype(self):
        return np.float64 if self.dtype == torch.float64 else np.float32

    def _local_d(self, x):
        """Slice a global d-vector to this rank's columns (COLS shards)."""
        if self.shard is not None and x.shape[0] == self.dim and self.device_matrix.d != self.dim:
            return x[self.shard.col_lo:self.shard.col_hi]
        return x

    def to_device(self, x, copy=False):
        """Device d-vector (local block of it in a column-sharded run)."""
        if isinstance(x, torch.Tensor):
            t = x.to(device=self.device, dtype=self.dtype)
            t = self._local_d(t)
            return t.clone().contiguous() if copy else t.contiguous()
        x = np.asarray(x)
        if sp_issparse(x):
            x = x.toarray().ravel()
        x = self._local_d(np.ascontiguousarray(x, dtype=self._np_dtype()))
        return torch.from_numpy(np.ascontiguousarray(x)).to(self.device)

    def to_host(self, x):
        return x.detach().to("cpu").numpy().copy() if isinstance(x, torch.Tensor) else np.array(x)

    def copy_vector(self, x):
        return x.clone() if isinstance(x, torch.Tensor) else copy.deepcopy(x)

    def norm_diff(self, a, b=None):
        """||a - b||_2 on the device (optimizer.py:110; all ranks in a sharded run)."""
        a = self.to_device(a)
        b = None if b is None else self.to_device(b)
        return self.device_matrix.diff_norm(a, b, space=_lib.KRCN_SPACE_D)

    def norm(self, x):
        return self.norm_diff(x)

    def any_rank(self, flag):
        """Rank-wide OR of a host flag (keeps SPMD loops in lockstep)."""
        if self.shard is None or self.shard.comm is None or self.shard.world == 1:
            return bool(flag)
        return self.shard.comm.any(flag)

    # ------------------------------------------------------- Ax / weights
    def reset(self):
        """loss.py:283-286."""
        self.reuse = False
        self.x_last = 0.0
        self._mat_vec_prod = None
        self._cache_x = self._cache_np = None
        self._w = None

    def _cached(self, x):
        if not self.store_mat_vec_prod or self._mat_vec_prod is None:
            return False
        if isinstance(x, torch.Tensor):
            return x is self._cache_x and x._version == self._cache_ver
        return self._cache_np is not None and np.array_equal(np.asarray(x), self._cache_np)

    def _device_Ax(self, x):
        if self._cached(x):
            return self._mat_vec_prod
        xd = self.to_device(x)
        Ax = self.device_matrix.matvec(xd)
        if self.store_mat_vec_prod:
            self._mat_vec_prod = Ax
            self._w = None
            if isinstance(x, torch.Tensor):
                self._cache_x, self._cache_ver, self._cache_np = x, x._version, None
            else:
                self._cache_x, self._cache_ver = None, None
                self._cache_np = np.array(x, copy=True)
            self.x_last = x
        return Ax

    def _weights_for(self, x):
        Ax = self._device_Ax(x)
        if self.store_mat_vec_prod and Ax is self._mat_vec_prod:
            if self._w is None:
                self._w = self.device_matrix.weights(Ax)
            return self._w
        return self.device_matrix.weights(Ax)

    def mat_vec_product(self, x):
        """Ax (loss.py:266-277); numpy in -> numpy out."""
        Ax = self._device_Ax(x)
        return Ax if isinstance(x, torch.Tensor) else self.to_host(Ax)

    # --------------------------------------------------------- oracle calls
    def _value(self, x):
        """mean((1-b) Ax - logsig(Ax)) + l2/2 ||x||^2 (loss.py:215-220)."""
        Ax = self._device_Ax(x)
        val = self.device_matrix.loss_mean(Ax, self._b_dev)
        if self.l2 != 0:
            val = val + self.l2 / 2 * self.norm_diff(x) ** 2
        return val

    def gradient(self, x):
        """X^T (expit(Ax) - b) / n (+ l2 x) (loss.py:223-232)."""
        Ax = self._device_Ax(x)
        xd = self.to_device(x) if self.l2 != 0 else None
        g = self.device_matrix.gradient(Ax, self._b_dev, xd, float(self.l2))
        return g if isinstance(x, torch.Tensor) else self.to_host(g)

    def hess_vec_prod(self, x, v, grad_dif=False, eps=None):
        """X^T (w * X v) / n + l2 v with w = s(1-s), s = expit(Ax) (loss.py:289-302)."""
        if grad_dif:
            gx = self.gradient(x)
            return (self.gradient(x + eps * v) - gx) / eps
        w = self._weights_for(x)
        y = self.device_matrix.hvp(w, self.to_device(v), l2=float(self.l2))
        return y if isinstance(v, torch.Tensor) else self.to_host(y)

    def hess_operator(self, x):
        return HessianOperator(self, x)

    # -------------------------------------------------- out-of-scope pieces
    def hessian(self, x):
        raise NotImplementedError("dense Hessian (full CRN, loss.py:249-255) is outside the device hot path")

    def partial_gradient(self, x, I):
        raise NotImplementedError("SSCN partial gradient (loss.py:234-247) is outside the device hot path")

    def partial_hessian(self, x, I):
        raise NotImplementedError("SSCN partial Hessian (loss.py:257-264) is outside the device hot path")

    def update_mat_vec_product(self, Ax, delta, I):
        raise NotImplementedError("SSCN Ax update (loss.py:279-281) is outside the device hot path")

    @property
    def smoothness(self):
        raise NotImplementedError("smoothness estimates (loss.py:308-337) are outside the device hot path; "
                                  "pass reg_coef explicitly")

    @property
    def hessian_lipschitz(self):
        raise NotImplementedError("hessian_lipschitz (loss.py:339-347) is outside the device hot path; "
                                  "pass reg_coef explicitly, as cubic_newton.py:67 does")

    @staticmethod
    def inner_prod(x, y):
        return x @ y

    @staticmethod
    def outer_prod(x, y):
        return np.outer(x, y)

    @staticmethod
    def is_equal(x, y):
        """loss.py:361-375 for dense inputs."""
        if x is None:
            return y is None
        if y is None:
            return False
        return np.array_equal(x, y)


def sp_issparse(x):
    import scipy.sparse as sp
    return sp.issparse(x)
