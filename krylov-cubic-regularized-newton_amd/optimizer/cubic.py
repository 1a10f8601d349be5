"""Krylov cubic-regularized Newton on the GPU (drop-in for optimizer/cubic.py).

Hot path (north_star): `Lanczos` + the logistic HVP run as hand-written gfx950
kernels through libkrcn; the recurrence's control state (alpha, beta, the
absolute 1e-6 breakdown test) stays on the device and only the m alphas / m-1
betas come back.  The m x m tridiagonal cubic subproblem (`cubic_solver_root`)
stays on the host, exactly as in the reference.

Reference: optimizer/cubic.py — cubic_solver_root :40-75, Lanczos :77-111,
Cubic_Krylov_LS :238-319.  Cubic_LS (:115-235) and SSCN (:321-408) are
comparison methods outside the hot path: importable, not runnable here.
"""
from __future__ import annotations

import numpy as np
import numpy.linalg as la
import scipy.sparse as sp
import torch
from scipy.linalg import solve
from scipy.optimize import root_scalar
from scipy.sparse.linalg import spsolve

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


def Lanczos(A, v, m=10, reorth=False, tol=1e-6, V=None):
    """m-step three-term Lanczos (cubic.py:77-111), on the GPU.

    A must be the device Hessian operator of a LogisticRegression
    (`loss.hess_operator(x)`) — the reference passes `lambda v:
    loss.hess_vec_prod(x, v)`, which cannot run on the device.  v: the start
    vector (numpy or device tensor).  Returns (V, alphas, betas, beta) like the
    reference: V is a (d, m_eff) device view (column j = basis vector j, backed
    by a row-major m x d buffer), alphas / betas numpy arrays after the
    reference's truncation rule, beta the last computed norm.
    reorth=True adds CGS2 full reorthogonalisation (not in the reference)."""
    if not isinstance(A, HessianOperator):
        raise TypeError("Lanczos needs a device operator: pass loss.hess_operator(x) "
                        "(there is no CPU path)")
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
                 reorth=False, breakdown_tol=1e-6, **kwargs):
        super().__init__(*args, **kwargs)
        self.solver_it = 0
        self.subspace_dim = subspace_dim
        self.solver_eps = solver_eps
        self.beta = beta
        self.r0 = 0.1
        self.value = None
        self.reorth = reorth
        self.breakdown_tol = breakdown_tol
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
        s_new, solver_it, r0_new, model_decrease = cubic_solver_root(
            self.grad, self.hess, reg_coef, epsilon=self.solver_eps, r0=self.r0)
        x_new = X.basis_combine(V, s_new, self.x)
        value_new = loss.value(x_new)
        trials = 0
        while value_new > self.value - model_decrease and trials < 20:
            reg_coef = reg_coef / self.beta
            s_new, solver_it, r0_new, model_decrease = cubic_solver_root(
                self.grad, self.hess, reg_coef, epsilon=self.solver_eps, r0=self.r0)
            x_new = X.basis_combine(V, s_new, self.x)
            value_new = loss.value(x_new)
            trials += 1
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


class Cubic_LS(Optimizer):
    """Full-space CRN (cubic.py:115-235): a comparison method outside the
    Krylov hot path.  Importable for drop-in compatibility; step() raises."""

    def __init__(self, reg_coef=None, cubic_solver="CG", solver_it_max=100, solver_eps=1e-8,
                 beta=0.5, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.reg_coef, self.cubic_solver = reg_coef, cubic_solver
        self.solver_it_max, self.solver_eps, self.beta = solver_it_max, solver_eps, beta
        self.solver_it, self.r0, self.value = 0, 0.1, None

    def step(self):
        raise NotImplementedError("Cubic_LS is outside the device hot path (SURVEY.md §2)")


class SSCN(Optimizer):
    """Stochastic subspace cubic Newton (cubic.py:321-408): a comparison method
    outside the Krylov hot path.  Importable; step() raises."""

    def __init__(self, reg_coef=None, subspace_dim=100, solver_eps=1e-8, beta=0.5, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.reg_coef, self.subspace_dim, self.solver_eps, self.beta = reg_coef, subspace_dim, solver_eps, beta
        self.solver_it, self.r0, self.value = 0, 0.1, None

    def step(self):
        raise NotImplementedError("SSCN is outside the device hot path (SURVEY.md §2)")
