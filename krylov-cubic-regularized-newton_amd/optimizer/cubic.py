"""Krylov cubic-regularized Newton on the GPU (drop-in for optimizer/cubic.py).

Hot path (north_star): `Lanczos` + the logistic HVP run as hand-written gfx950
kernels through libkrcn; the recurrence's control state (alpha, beta, the
absolute 1e-6 breakdown test) stays on the device and only the m alphas / m-1
betas come back.  The m x m tridiagonal cubic subproblem stays on the host, as
in the reference, but as O(m) tridiagonal LDL^T solves (LAPACK dpttrf/dpttrs)
instead of a dense Cholesky per Newton evaluation (cubic_solver_root_tridiag).

The comparison methods of cubic_newton.py run on the same device kernels:
Cubic_LS (full-space CRN: "CG" solves with device conjugate gradients on the
HVP, krcn_cg_solve; "full" factors the dense Hessian built from HVPs) and SSCN
(coordinate subspaces: partial gradient / Hessian and the incremental Ax
update on the device).  Lanczos also accepts any callable operator.

Reference: optimizer/cubic.py — cubic_solver_root :40-75, Lanczos :77-111,
Cubic_LS :115-235, Cubic_Krylov_LS :238-319, SSCN :321-408.
"""
from __future__ import annotations

import copy
import warnings

import numpy as np
import numpy.linalg as la
import scipy.sparse as sp
import torch
from scipy.linalg import lapack, solve
from scipy.optimize import root_scalar
from scipy.sparse.linalg import spsolve

from krcn.vec import VecContext

from .loss import HessianOperator
from .optimizer import Optimizer


def cubic_solver_root(g, H, M, it_max=100, epsilon=1e-8, r0=0.1):
    """argmin_s <g,s> + 1/2 <s,Hs> + M/3 ||s||^3 on the host (cubic.py:40-75).

    Newton's method on phi(lam) = lam^2 - M^2 ||s(lam)||^2, s(lam) = -(H + lam I)^{-1} g
    (Cartis, Gould & Toint 2011, §6.1).  Returns (s, newton iterations, lam,
    model decrease).  The arithmetic is written term for term like the
    reference so the host trajectory is bit-identical given identical T."""
    g = np.asarray(g)
    m = len(g)
    if sp.issparse(H) and m >= 500:
        eye = sp.eye(m)

        def shifted_solve(lam, rhs):
            return spsolve(H + lam * eye, rhs)
    else:
        Hd = H.toarray() if sp.issparse(H) else H
        eye = np.eye(m)

        def shifted_solve(lam, rhs):
            return solve(Hd + lam * eye, rhs, assume_a="pos")

    def phi(lam):
        s_lam = -shifted_solve(lam, g)
        return lam ** 2 - M ** 2 * np.linalg.norm(s_lam) ** 2

    def dphi(lam):
        s_lam = -shifted_solve(lam, g)
        dnorm2 = -2 * np.dot(s_lam, shifted_solve(lam, s_lam))
        return 2 * lam - M ** 2 * dnorm2

    sol = root_scalar(phi, fprime=dphi, x0=r0, method="newton", maxiter=it_max, xtol=epsilon)
    lam = sol.root
    s = -shifted_solve(lam, g)
    ns = la.norm(s)
    model_decrease = lam / 2 * ns ** 2 - M / 3 * ns ** 3 - np.dot(g, s) / 2
    return s, sol.iterations, lam, model_decrease


def cubic_solver_root_tridiag(g, alphas, betas, M, it_max=100, epsilon=1e-8, r0=0.1):
    """cubic_solver_root for H = tridiag(betas, alphas, betas), the Krylov
    subspace Hessian of Cubic_Krylov_LS (cubic.py:278-285).

    Same Newton iteration on phi(lam) = lam^2 - M^2 ||s(lam)||^2 (root_scalar,
    same x0 / xtol / maxiter) and the same closing expressions as
    cubic_solver_root, but each shifted solve (T + lam I) s = rhs is a
    tridiagonal LDL^T factorisation (LAPACK dpttrf, O(m)) shared by every solve
    at the same lam, instead of a dense Cholesky (solve(assume_a='pos'),
    O(m^3)) per solve.  A shift that leaves T + lam I indefinite raises
    LinAlgError, as the dense positive-definite solve does.  Results agree with
    the dense path to rounding (tests/test_host_logic.py)."""
    g = np.asarray(g, dtype=np.float64)
    al = np.asarray(alphas, dtype=np.float64)
    be = np.asarray(betas, dtype=np.float64)
    if len(al) != len(g) or len(be) != max(len(g) - 1, 0):
        raise ValueError("alphas must have len(g) entries and betas len(g) - 1")
    fact = {}
    be_arg = be if len(be) else np.zeros(1)   # LAPACK's e has max(m - 1, 1) slots

    def shifted_solve(lam, rhs):
        f = fact.get(lam)
        if f is None:
            dd, ee, info = lapack.dpttrf(al + lam, be_arg)
            if info != 0:
                raise la.LinAlgError("T + lam I is not positive definite")
            fact.clear()
            fact[lam] = f = (dd, ee)
        x, info = lapack.dpttrs(f[0], f[1], rhs)
        if info != 0:
            raise la.LinAlgError(f"dpttrs failed (info {info})")
        return x

    def phi(lam):
        s_lam = -shifted_solve(lam, g)
        return lam ** 2 - M ** 2 * np.linalg.norm(s_lam) ** 2

    def dphi(lam):
        s_lam = -shifted_solve(lam, g)
        dnorm2 = -2 * np.dot(s_lam, shifted_solve(lam, s_lam))
        return 2 * lam - M ** 2 * dnorm2

    sol = root_scalar(phi, fprime=dphi, x0=r0, method="newton", maxiter=it_max, xtol=epsilon)
    lam = sol.root
    s = -shifted_solve(lam, g)
    ns = la.norm(s)
    model_decrease = lam / 2 * ns ** 2 - M / 3 * ns ** 3 - np.dot(g, s) / 2
    return s, sol.iterations, lam, model_decrease


def _lanczos_callable(A, v, m, tol):
    """cubic.py:77-111 over a plain callable A, every vector operation on the
    device (krcn_vctx kernels): A is called once per step.  A numpy v means a
    numpy operator (called with host vectors, results uploaded) and returns V
    as a numpy (d, m_eff) array; a device tensor v keeps A's traffic on the
    device and returns a (d, m_eff) device view."""
    numpy_mode = not isinstance(v, torch.Tensor)
    if numpy_mode:
        if not torch.cuda.is_available():
            raise RuntimeError("Lanczos runs on the GPU (no CPU path exists)")
        dev = torch.device("cuda", torch.cuda.current_device())
        vd = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(dev)
    else:
        vd = v.detach().contiguous()
        dev = vd.device
    ctx = VecContext.for_device(dev)
    d = vd.numel()

    def apply(q):
        y = A(q.cpu().numpy() if numpy_mode else q)
        if isinstance(y, torch.Tensor):
            return y.to(device=dev, dtype=vd.dtype).contiguous()
        return torch.from_numpy(np.ascontiguousarray(np.asarray(y).ravel(), dtype=np.float64)).to(dev, vd.dtype)

    V = torch.zeros((m, d), dtype=vd.dtype, device=dev)     # cubic.py:88 (zeros: the quirk column)
    ctx.div(vd, np.sqrt(ctx.dot(vd, vd)), out=V[0])          # cubic.py:85-89
    alphas = np.zeros(m)
    betas = np.zeros(max(m - 1, 0))
    beta = 0.0
    v_pre = None
    vj = V[0]
    z = torch.empty_like(vd)
    j = 0
    for j in range(m - 1):                                   # cubic.py:92-103
        y = apply(vj)
        alpha, beta = ctx.lz_step(y, vj, v_pre, beta, z)
        alphas[j] = alpha
        if np.abs(beta) < tol:
            break
        betas[j] = beta
        v_pre = vj
        ctx.div(z, beta, out=V[j + 1])
        vj = V[j + 1]
    m_eff = m
    if m > 1 and j < m - 2:                                  # cubic.py:105-108
        m_eff = j + 1
        alphas = alphas[:j + 1]
        betas = betas[:j]
    alphas[-1] = ctx.dot(vj, apply(vj))                       # cubic.py:109
    Vt = V[:m_eff].T
    return (Vt.cpu().numpy() if numpy_mode else Vt), alphas, betas, beta


def Lanczos(A, v, m=10, reorth=False, tol=1e-6, V=None):
    """m-step three-term Lanczos (cubic.py:77-111), on the GPU.

    A: the device Hessian operator of a LogisticRegression
    (`loss.hess_operator(x)`: the fused device recurrence, krcn_lanczos), or any
    callable v -> A v, such as the reference's `lambda v: loss.hess_vec_prod(x,
    v)` (cubic.py:273): it is called once per step and the recurrence's vector
    work runs on the device (krcn_lz_ext_step).  v: the start vector (numpy or
    device tensor).  Returns (V, alphas, betas, beta) like the reference: V is
    (d, m_eff) — a device view for the operator / a device v, a numpy array for
    a numpy v with a callable —, alphas / betas numpy arrays after the
    reference's truncation rule, beta the last computed norm.
    reorth=True adds CGS2 full reorthogonalisation (not in the reference; fused
    operator only)."""
    if not isinstance(A, HessianOperator):
        if not callable(A):
            raise TypeError("Lanczos needs a callable operator or loss.hess_operator(x)")
        if reorth:
            raise NotImplementedError("reorth=True needs the fused device operator loss.hess_operator(x)")
        if V is not None:
            raise ValueError("V is only accepted with the fused device operator")
        return _lanczos_callable(A, v, int(m), tol)
    X = A.X
    g = A.loss.to_device(v)
    Vb, alphas, betas, info = X.lanczos(A.w, g, m, reorth=reorth, tol=tol, l2=A.l2, V=V)
    return Vb[:info.m_eff].T, alphas, betas, info.beta_last


class Cubic_Krylov_LS(Optimizer):
    """Krylov cubic regularized Newton with line search (cubic.py:238-319).

    reg_coef: cubic regularization estimate (required: the Lipschitz estimate
    of the reference's default is outside the hot path); subspace_dim: Krylov
    dimension m; solver_eps: tolerance of the host subproblem; beta:
    backtracking factor.  Build-only extras: reorth (CGS2 in Lanczos), tol
    (absolute breakdown threshold, 1e-6 as cubic.py:98)."""

    def __init__(self, reg_coef=None, subspace_dim=100, solver_eps=1e-8, beta=0.5, *args,
                 reorth=False, breakdown_tol=1e-6, dense_subproblem=False, **kwargs):
        super().__init__(*args, **kwargs)
        self.solver_it = 0
        self.subspace_dim = subspace_dim
        self.solver_eps = solver_eps
        self.beta = beta
        self.r0 = 0.1
        self.value = None
        self.reorth = reorth
        self.breakdown_tol = breakdown_tol
        self.dense_subproblem = dense_subproblem
        self.reg_coef = self.loss.hessian_lipschitz if reg_coef is None else reg_coef
        self._V = None
        self.last_lanczos = None

    def _basis(self):
        X = self.loss.device_matrix
        m = self.subspace_dim
        if self._V is None or self._V.shape != (m, X.d):
            self._V = torch.empty((m, X.d), dtype=X.dtype, device=X.device)
        return self._V

    def step(self):
        """One Krylov-CRN step (cubic.py:265-309): grad -> Lanczos -> host cubic
        subproblem over T -> x + V s -> backtracking (at most 20 trials)."""
        loss = self.loss
        X = loss.device_matrix
        if self.value is None:
            self.value = loss.value(self.x)
        grad = loss.gradient(self.x)
        op = loss.hess_operator(self.x)
        V, alphas, betas, info = X.lanczos(op.w, grad, self.subspace_dim, reorth=self.reorth,
                                           tol=self.breakdown_tol, l2=op.l2, V=self._basis())
        self.last_lanczos = info
        self.hess = np.diag(alphas) + np.diag(betas, -1) + np.diag(betas, 1)
        e1 = np.zeros(len(alphas))
        e1[0] = 1
        self.grad = info.gnorm * e1
        reg_coef = self.reg_coef * self.beta
        s_new, solver_it, r0_new, model_decrease = self._subproblem(alphas, betas, reg_coef)
        x_new = X.basis_combine(V, s_new, self.x)
        value_new = loss.value(x_new)
        trials = 0
        while value_new > self.value - model_decrease and trials < 20:
            reg_coef = reg_coef / self.beta
            s_new, solver_it, r0_new, model_decrease = self._subproblem(alphas, betas, reg_coef)
            x_new = X.basis_combine(V, s_new, self.x)
            value_new = loss.value(x_new)
            trials += 1
        self.x = x_new
        self.reg_coef = reg_coef
        self.value = value_new
        self.r0 = r0_new
        self.solver_it += solver_it

    def _subproblem(self, alphas, betas, reg_coef):
        """The m x m cubic subproblem over T = tridiag(betas, alphas, betas)
        (cubic.py:285-286): O(m) tridiagonal solves, or the reference's dense
        solver with dense_subproblem=True."""
        if self.dense_subproblem:
            return cubic_solver_root(self.grad, self.hess, reg_coef, epsilon=self.solver_eps, r0=self.r0)
        return cubic_solver_root_tridiag(self.grad, alphas, betas, reg_coef, epsilon=self.solver_eps,
                                         r0=self.r0)

    def init_run(self, *args, **kwargs):
        super().init_run(*args, **kwargs)
        self.trace.solver_its = [0]
        self.loss.reset()

    def update_trace(self):
        super().update_trace()
        self.trace.solver_its.append(self.solver_it)


class Cubic_LS(Optimizer):
    """Full-space cubic regularized Newton with line search (cubic.py:115-235;
    Nesterov & Polyak 2006), on the device kernels.

    cubic_solver="CG": every linear solve of the subproblem's Newton iteration
    is device conjugate gradients on v -> hess_vec_prod(x, v) + lam v
    (krcn_cg_solve, scipy cg's loop and stopping rule with rtol = solver_eps,
    the reference's `cg(..., tol=epsilon)`, cubic.py:152-182).
    cubic_solver="full": the dense Hessian (loss.hessian, built from HVPs on the
    device) goes to the host subproblem solver, cubic.py:184-188.
    Arguments and trace as the reference."""

    def __init__(self, reg_coef=None, cubic_solver="CG", solver_it_max=100, solver_eps=1e-8,
                 beta=0.5, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.solver_it = 0
        self.solver_it_max = solver_it_max
        self.solver_eps = solver_eps
        self.beta = beta
        self.r0 = 0.1
        self.residuals = []
        self.value = None
        self.cg_iterations = 0          # device CG iterations (not in the reference's trace)
        self.cg_unconverged = 0         # CG solves that hit maxiter (scipy's info > 0)
        self.reg_coef = self.loss.hessian_lipschitz if reg_coef is None else reg_coef
        if cubic_solver == "CG":
            self.cubic_solver = self.cubic_solver_root_CG
        elif cubic_solver == "full":
            self.cubic_solver = self.cubic_solver_root_full
        else:
            print("Error: cubic_solver not recognized")

    def cubic_solver_root_CG(self, M, it_max=100, epsilon=1e-8, r0=0.1):
        """cubic_solver_root with every (H + lam I)^{-1} applied by device CG
        (cubic.py:152-182).  CG is linear in its right-hand side and IEEE
        negation is exact, so solving with g and negating reproduces the
        reference's cg(H_lambda, -g) without materialising -g.  Returns
        (s, newton iterations, lam, model decrease); s is a device d-vector."""
        loss = self.loss
        X = loss.device_matrix
        g = self.grad
        w = loss._weights_for(self.x)
        l2 = float(loss.l2)
        sol_cache = {}
        # a relative residual below ~10 ulp of the working precision is out of
        # reach: asked for 1e-8 in fp32, every solve would run its 10 d
        # iterations without ever stopping (fp64 keeps the reference's tol)
        rtol = max(float(epsilon), 10.0 * float(torch.finfo(X.dtype).eps))

        def cg(lam, rhs):
            x, info = X.cg_solve(w, rhs, shift=l2 + lam, rtol=rtol)
            self.cg_iterations += info.iterations
            if not info.converged:
                self.cg_unconverged += 1
                if self.cg_unconverged == 1:
                    warnings.warn(f"device CG stopped at maxiter = {info.iterations} with ||r|| = "
                                  f"{info.residual_norm:.3e} (rtol {rtol:.1e}); counted in cg_unconverged")
            return x

        def neg_s(lam):          # -s(lam) = (H + lam I)^{-1} g
            y = sol_cache.get(lam)
            if y is None:
                sol_cache.clear()
                sol_cache[lam] = y = cg(lam, g)
            return y

        def func(lam):
            return lam ** 2 - M ** 2 * X.diff_norm(neg_s(lam)) ** 2

        def grad(lam):
            y = neg_s(lam)                   # s = -y; H_lam^{-1} s = -H_lam^{-1} y
            phi_lam_grad = -2 * X.dot(y, cg(lam, y))
            return 2 * lam - M ** 2 * phi_lam_grad

        sol = root_scalar(func, fprime=grad, x0=r0, method="newton", maxiter=it_max, xtol=epsilon)
        r = sol.root
        y = cg(r, g)
        norm_s = X.diff_norm(y)
        model_decrease = r / 2 * norm_s ** 2 - M / 3 * norm_s ** 3 + X.dot(g, y) / 2
        s = VecContext.for_device(X.device).axpy(-1.0, y, torch.zeros_like(y))
        return s, sol.iterations, r, model_decrease

    def cubic_solver_root_full(self, M, it_max=100, epsilon=1e-8, r0=0.1):
        """The host subproblem over the dense Hessian (cubic.py:184-188)."""
        g = self.loss.to_host(self.grad)
        return cubic_solver_root(g, self.hess, M, it_max=it_max, epsilon=epsilon, r0=r0)

    def _add(self, s):
        s = self.loss.to_device(s)
        return VecContext.for_device(self.loss.device).axpy(1.0, s, self.x)

    def step(self):
        """cubic.py:190-224: gradient, (dense Hessian), cubic subproblem,
        x + s, backtracking on reg_coef until sufficient decrease."""
        loss = self.loss
        if self.value is None:
            self.value = loss.value(self.x)
        self.grad = loss.gradient(self.x)
        if self.cubic_solver == self.cubic_solver_root_full:
            self.hess = loss.hessian(self.x)
        if loss.norm(self.grad) < self.tolerance:
            return
        reg_coef = self.reg_coef * self.beta
        s_new, solver_it, r0_new, model_decrease = self.cubic_solver(
            reg_coef, self.solver_it_max, self.solver_eps, r0=self.r0)
        x_new = self._add(s_new)
        value_new = loss.value(x_new)
        while value_new > self.value - model_decrease:
            reg_coef = reg_coef / self.beta
            s_new, solver_it, r0_new, model_decrease = self.cubic_solver(
                reg_coef, self.solver_it_max, self.solver_eps, r0=self.r0)
            x_new = self._add(s_new)
            value_new = loss.value(x_new)
        self.x = x_new
        self.reg_coef = reg_coef
        self.value = value_new
        self.r0 = r0_new
        self.solver_it += solver_it

    def init_run(self, *args, **kwargs):
        super().init_run(*args, **kwargs)
        self.trace.solver_its = [0]
        self.loss.reset()

    def update_trace(self):
        super().update_trace()
        self.trace.solver_its.append(self.solver_it)


class SSCN(Optimizer):
    """Stochastic subspace cubic Newton, coordinate version (cubic.py:321-408;
    Hanzely et al. 2020, §7.1), on the device kernels: the coordinate gradient
    and Hessian (loss.partial_gradient / partial_hessian), the coordinate
    update of x and the incremental Ax update (loss.update_mat_vec_product)
    run on the GPU; the m x m subproblem on the host, as in the reference."""

    def __init__(self, reg_coef=None, subspace_dim=100, solver_eps=1e-8, beta=0.5, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.reg_coef = reg_coef
        self.solver_it = 0
        self.subspace_dim = subspace_dim
        self.solver_eps = solver_eps
        self.beta = beta
        self.r0 = 0.1
        self.residuals = []
        self.value = None
        self.tolerance = 0
        if reg_coef is None:
            self.reg_coef = self.loss.hessian_lipschitz
        self.reuse = False

    def _coordinate_step(self, I_dev, s_sub):
        x_new = self.x.clone()
        x_new[I_dev] = self.x[I_dev] + torch.from_numpy(np.asarray(s_sub, dtype=np.float64)).to(
            self.x.device, self.x.dtype)
        return x_new

    def step(self):
        """cubic.py:349-399."""
        loss = self.loss
        if self.value is None:
            self.value = loss.value(self.x)
        I = self.rng.choice(self.dim, size=self.subspace_dim, replace=False)
        I_dev = torch.from_numpy(np.asarray(I, dtype=np.int64)).to(self.x.device)
        self.grad = loss.partial_gradient(self.x, I)
        self.hess = loss.partial_hessian(self.x, I)
        reg_coef = max(self.reg_coef * self.beta, np.finfo(float).eps)
        Ax = copy.deepcopy(loss._mat_vec_prod)
        s_new_sub, solver_it, r0_new, model_decrease = cubic_solver_root(
            self.grad, self.hess, reg_coef, r0=self.r0, epsilon=np.finfo(float).eps)
        x_new = self._coordinate_step(I_dev, s_new_sub)
        loss.update_mat_vec_product(Ax, s_new_sub, I)
        value_new = loss.value(x_new)
        while value_new > self.value - model_decrease:
            reg_coef = reg_coef / self.beta
            s_new_sub, solver_it, r0_new, model_decrease = cubic_solver_root(
                self.grad, self.hess, reg_coef, r0=self.r0, epsilon=np.finfo(float).eps)
            x_new = self._coordinate_step(I_dev, s_new_sub)
            loss.update_mat_vec_product(Ax, s_new_sub, I)
            value_new = loss.value(x_new)
        self.x = x_new
        self.reg_coef = reg_coef
        self.value = value_new
        self.r0 = r0_new
        self.solver_it += solver_it

    def init_run(self, *args, **kwargs):
        super().init_run(*args, **kwargs)
        self.trace.solver_its = [0]
        self.loss.reset()

    def update_trace(self):
        super().update_trace()
        self.trace.solver_its.append(self.solver_it)
