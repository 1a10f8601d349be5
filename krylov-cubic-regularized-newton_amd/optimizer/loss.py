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

The comparison methods' pieces (dense `hessian`, the SSCN `partial_*` methods,
`update_mat_vec_product`) and the smoothness estimates run on the device
kernels for unsharded problems (they raise NotImplementedError on a shard);
l1 / prox regularizers are out of scope and raise
NotImplementedError.
"""
from __future__ import annotations

import copy
import warnings

import numpy as np
import torch

import krcn
from krcn import _lib
from krcn.labels import labels01 as _labels01


class _PinnedArena:
    """Pinned host storage for trace checkpoints, allocated in chunks of
    several d-vectors (about 64 MB each) so a checkpoint is one async copy
    rather than a pinned allocation plus a synchronous one."""

    _CHUNK_BYTES = 64 << 20

    def __init__(self):
        self.chunk = None
        self.used = 0

    def take(self, numel, dtype):
        c = self.chunk
        if c is None or self.used == c.shape[0] or c.shape[1] != numel or c.dtype != dtype:
            per = max(1, self._CHUNK_BYTES // max(1, numel * torch.empty((), dtype=dtype).element_size()))
            self.chunk = torch.empty((per, numel), dtype=dtype, pin_memory=True)
            self.used = 0
        row = self.chunk[self.used]
        self.used += 1
        return row


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

    def to_host_async(self, x):
        """A checkpoint copy of x that does not wait for the device: an async
        D2H copy on the current stream into pinned host memory, returned as a
        numpy view of it.  The view holds x's value once the stream has passed
        the copy — every later Lanczos call synchronises the stream, and
        `sync()` does so explicitly (Optimizer.run calls it before returning)."""
        if not (isinstance(x, torch.Tensor) and x.is_cuda):
            return self.to_host(x)
        if not hasattr(self, "_arena"):
            self._arena = _PinnedArena()
        row = self._arena.take(x.numel(), x.dtype)
        row.copy_(x.detach().reshape(-1), non_blocking=True)
        return row.numpy()

    def sync(self):
        """Wait for the async checkpoint copies on this loss's device."""
        if getattr(self, "_arena", None) is not None and self._arena.used:
            torch.cuda.current_stream(self.device).synchronize()

    # ------------------------------------------------ stored iterates
    _DEV_ITER_CAP = 8 << 30   # device bytes of kept iterate copies, at most

    def keep_device_iterate(self, x):
        """A device copy of a trace iterate (Optimizer.update_trace), or None
        past the budget (min(8 GiB, a quarter of the device)); the copy's bytes
        return to the budget when the trace drops it.  The budget counts the
        GLOBAL d-vector, so every rank of a sharded run (whose local d differ
        in a column split) keeps copies of the same iterates and
        values_of_iterates issues the same collectives on all of them."""
        if not (isinstance(x, torch.Tensor) and x.is_cuda):
            return None
        nbytes = int(self.dim) * x.element_size()
        if not hasattr(self, "_dev_iter_bytes"):
            self._dev_iter_bytes = [0]
            # (hipMemGetInfo; torch.cuda.get_device_properties re-counts the
            # devices through amdsmi until torch has initialised, which failed
            # as "Invalid device id" with 8 virtual-rank threads asking at once)
            total = torch.cuda.mem_get_info(self.device)[1]
            self._dev_iter_cap = min(self._DEV_ITER_CAP, total // 4)
        if self._dev_iter_bytes[0] + nbytes > self._dev_iter_cap:
            return None
        c = x.detach().clone()
        import weakref
        self._dev_iter_bytes[0] += nbytes
        weakref.finalize(c, _release, self._dev_iter_bytes, nbytes)
        return c

    def values_of_iterates(self, xs, dev):
        """[self.value(x) for x in xs] (opt_trace.py:39-41) with the iterates
        that have device copies in `dev` (id(x) -> (x, copy)) evaluated by one
        krcn_loss_values submission; the rest, and the best-iterate tracking
        (loss.py:66-73: f_opt / x_opt updated in order), as the loop does."""
        idx = [i for i, x in enumerate(xs) if id(x) in dev and dev[id(x)][0] is x]
        vals = [None] * len(xs)
        if idx:
            cop = [dev[id(xs[i])][1] for i in idx]
            for i, v, c in zip(idx, self.device_matrix.loss_values(cop, self._b_dev), cop):
                vals[i] = v + self.l2 / 2 * self.norm_diff(c) ** 2 if self.l2 != 0 else v
        out = []
        for i, x in enumerate(xs):
            if vals[i] is None:
                out.append(self.value(x))
                continue
            v = vals[i]
            if v < self.f_opt:
                self.x_opt = x.clone() if isinstance(x, torch.Tensor) else copy.deepcopy(x)
                self.f_opt = v
            out.append(v)
        return out

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
        if self.reuse:            # SSCN keeps Ax current itself (loss.py:267, :279-281)
            return True
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

    # ------------------------------------- full-space CRN and SSCN pieces
    def _unit_columns(self, x, cols):
        """Columns `cols` of the Hessian at x as device tensors: H e_c by the
        device HVP (e_c one unit vector each; the l2 term lands on the diagonal)."""
        self._no_shards("the dense / coordinate Hessian")
        w = self._weights_for(x)
        X = self.device_matrix
        e = torch.zeros(self.dim, dtype=self.dtype, device=self.device)
        out = []
        for c in cols:
            e[int(c)] = 1.0
            out.append(X.hvp(w, e, l2=float(self.l2)))
            e[int(c)] = 0.0
        return out

    def _no_shards(self, what):
        if self.shard is not None:
            raise NotImplementedError(f"{what} is implemented for unsharded problems")

    def hessian(self, x):
        """Dense Hessian X^T diag(w) X / n + l2 I (loss.py:249-255), one device
        HVP per column; numpy (d, d), for the full-space CRN at small d."""
        cols = self._unit_columns(x, range(self.dim))
        return torch.stack(cols, dim=1).cpu().numpy().astype(np.float64)

    def partial_gradient(self, x, I):
        """Coordinates I of the gradient (loss.py:234-247): the device gradient
        (per-coordinate sums in row order, X^T of loss.py:239) gathered at I;
        numpy (len(I),)."""
        self._no_shards("partial_gradient")
        g = self.gradient(self.to_device(x))
        idx = torch.from_numpy(np.asarray(I, dtype=np.int64)).to(self.device)
        return g.index_select(0, idx).cpu().numpy().astype(np.float64)

    def partial_hessian(self, x, I):
        """The I x I block of the Hessian (loss.py:257-264): len(I) device HVPs
        on unit vectors, rows I kept; a scipy sparse (CSR) matrix like the
        reference's A_weighted @ A[:, I] / n + l2 eye."""
        import scipy.sparse as sp
        idx = torch.from_numpy(np.asarray(I, dtype=np.int64)).to(self.device)
        cols = [c.index_select(0, idx) for c in self._unit_columns(x, I)]
        return sp.csr_matrix(torch.stack(cols, dim=1).cpu().numpy().astype(np.float64))

    def update_mat_vec_product(self, Ax, delta, I):
        """Ax + A[:, I] delta becomes the cached product, reused for every x
        until reset() (loss.py:279-281, SSCN's incremental update): one device
        pass over X with delta scattered into a zero d-vector."""
        self._no_shards("update_mat_vec_product")
        from krcn.vec import VecContext
        dv = torch.zeros(self.dim, dtype=self.dtype, device=self.device)
        idx = torch.from_numpy(np.asarray(I, dtype=np.int64)).to(self.device)
        dv[idx] = torch.from_numpy(np.asarray(delta, dtype=np.float64)).to(self.device, self.dtype)
        AI = self.device_matrix.matvec(dv)
        # the reference starts the cache as zeros(n) (loss.py:283-286): with
        # store_mat_vec_prod=False SSCN hands back that never-written zero
        # vector (here: None) and the sum is never read (mat_vec_product
        # recomputes A x), so A[:, I] delta alone stands in for it
        self._mat_vec_prod = AI if Ax is None else VecContext.for_device(self.device).axpy(1.0, AI, Ax)
        self._w = None
        self.reuse = True

    # ------------------------------------------------- smoothness constants
    def _lambda_max_gram(self, m=64):
        """Largest eigenvalue of X^T X / n: the top Ritz value of a device
        Lanczos (CGS2-reorthogonalised) on v -> X^T (1 * X v) / n from a
        constant start vector, the eigenvalue svds(A, k=1)^2 / n refers to."""
        X = self.device_matrix
        ones_n = torch.ones(X.n, dtype=self.dtype, device=self.device)
        # the basis is m x d: at most 512 vectors and 1 GiB of them
        esz = torch.empty((), dtype=self.dtype).element_size()
        cap = max(1, min(512, self.dim, (1 << 30) // max(1, X.d * esz)))

        def top_ritz(v0, m):
            # the top Ritz pair of an m-step Lanczos, grown until its true
            # residual ||H y - theta y|| is below 1e-8 theta (a Ritz value is
            # only a lower bound on lambda_max until it has converged)
            while True:
                V, al, be, info = X.lanczos(ones_n, v0, m, reorth=True, tol=1e-14)
                T = np.diag(al) + np.diag(be, -1) + np.diag(be, 1)
                th, S = np.linalg.eigh(T)
                theta = float(th[-1])
                if info.breakdown or m >= cap:   # an invariant subspace: theta is exact in it
                    return theta, bool(info.breakdown)
                zero = torch.zeros(X.d, dtype=self.dtype, device=self.device)
                y = X.basis_combine(V, S[:, -1], zero)
                Hy = X.hvp(ones_n, y)
                res = X.diff_norm(Hy, (theta * y).contiguous())
                if res <= 1e-8 * abs(theta):
                    return theta, False
                m = min(2 * m, cap)

        m = max(1, min(int(m), self.dim))
        theta, invariant = top_ritz(torch.ones(X.d, dtype=self.dtype, device=self.device), m)
        if invariant and self.dim > 1:
            # the constant start spans an invariant subspace that may miss the
            # top eigenvector (mixed-sign features): restart at random, keep the max
            g = torch.Generator(device="cpu").manual_seed(self.seed)
            v1 = torch.randn(X.d, generator=g, dtype=torch.float64).to(self.device, self.dtype)
            theta = max(theta, top_ritz(v1, m)[0])
        return theta

    @property
    def smoothness(self):
        """L of the logistic loss (loss.py:308-320): 0.25 sigma_max(A)^2 / n + l2,
        or the Frobenius bound for n, d > 20000.  sigma_max^2 / n comes from the
        device Lanczos (the reference calls ARPACK's svds); ||A||_F^2 from a
        device dot of the values."""
        if getattr(self, "_smoothness", None) is not None:
            return self._smoothness
        self._no_shards("smoothness")
        X = self.device_matrix
        if self.dim > 20000 and self.n > 20000:
            warnings.warn("The matrix is too large to estimate the smoothness constant, so Frobenius "
                          "estimate is used instead.")
            from krcn.vec import VecContext
            fro2 = VecContext.for_device(self.device).dot(X.data, X.data)
            self._smoothness = 0.25 * fro2 / self.n + self.l2
        else:
            self._smoothness = 0.25 * self._lambda_max_gram() + self.l2
        return self._smoothness

    @property
    def hessian_lipschitz(self):
        """Lipschitz estimate of the Hessian, max ||a_i|| * max |third derivative|
        * ||A||^2 = (4 (L - l2)) max ||a_i|| / (6 sqrt 3) (loss.py:339-347)."""
        if getattr(self, "_hessian_lipschitz", None) is not None:
            return self._hessian_lipschitz
        import scipy.sparse as sp
        A = sp.csr_matrix(self.A)
        lens = np.diff(A.indptr)
        sq = np.add.reduceat(A.data ** 2, A.indptr[:-1][lens > 0]) if A.nnz else np.zeros(1)
        a_max = float(np.sqrt(sq.max()))
        A_norm = (self.smoothness - self.l2) * 4
        self._hessian_lipschitz = A_norm * a_max / (6 * np.sqrt(3))
        return self._hessian_lipschitz

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


def _release(counter, nbytes):
    counter[0] -= nbytes


def sp_issparse(x):
    import scipy.sparse as sp
    return sp.issparse(x)
