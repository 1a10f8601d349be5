"""CPU oracle for the Krylov-CRN hot path — TEST INFRASTRUCTURE ONLY.

This module restates, in numpy/scipy, the reference algorithms the GPU path
must reproduce (Raymond30/Krylov-Cubic-Regularized-Newton @ 2025-01-17):
  optimizer/loss.py   logsig :161-176, label map :189-207, _value :215-220,
                      gradient :223-232, mat_vec_product :266-277,
                      hess_vec_prod :289-302
  optimizer/cubic.py  cubic_solver_root :40-75, Lanczos :77-111,
                      Cubic_Krylov_LS.step :265-309
It uses the same third-party calls the reference uses (scipy csr_matvec via
`A @ v`, csc_matvec via `A.T @ u`, scipy.special.expit, numpy dot/norm,
scipy.linalg.solve(assume_a='pos'), root_scalar(method='newton')).

Pinning: tests/test_oracle_golden.py checks every function here against golden
vectors that tests/golden/make_golden.py produced by importing the reference
itself in the build container (numba stubbed: only loss.logsig is @njit, and
it is plain numpy).  See DESIGN.md "Oracle".

Who may import this: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — as the checker / the timed CPU baseline only.  The product
package (krylov-cubic-regularized-newton_amd/) never imports it.
"""
from __future__ import annotations

import numpy as np
import numpy.linalg as la
import scipy.special
from scipy.linalg import solve
from scipy.optimize import root_scalar


# ----------------------------------------------------------- loss.py
def logsig(x):
    """Piecewise log-sigmoid (loss.py:161-176)."""
    out = np.zeros_like(x)
    i0 = x < -33
    out[i0] = x[i0]
    i1 = (x >= -33) & (x < -18)
    out[i1] = x[i1] - np.exp(x[i1])
    i2 = (x >= -18) & (x < 37)
    out[i2] = -np.log1p(np.exp(-x[i2]))
    i3 = x >= 37
    out[i3] = -np.exp(-x[i3])
    return out


def labels01(b):
    """{1,2} -> {0,1}, {-1,1} -> {0,1}, other pairs -> (b == b[0]) (loss.py:189-207)."""
    b = np.asarray(b)
    u = np.unique(b)
    if len(u) > 2:
        raise ValueError("more than two classes")
    if len(u) == 2 and (u != [0, 1]).any():
        if (u == [1, 2]).all():
            return b - 1
        if (u == [-1, 1]).all():
            return (b + 1) / 2
        return 1.0 * (b == b[0])
    return b


def mat_vec_product(A, x):
    """A @ x (loss.py:270)."""
    return np.asarray(A @ x).ravel()


def value(A, b01, x, l2=0.0):
    """mean((1-b) Ax - logsig(Ax)) + l2/2 ||x||^2 (loss.py:215-220)."""
    Ax = mat_vec_product(A, x)
    reg = 0
    if l2 != 0:
        reg = l2 / 2 * la.norm(x) ** 2
    return np.mean(np.multiply(1 - b01, Ax) - logsig(Ax)) + reg


def gradient(A, b01, x, l2=0.0):
    """A^T (expit(Ax) - b) / n (+ l2 x) (loss.py:223-232)."""
    n = A.shape[0]
    act = scipy.special.expit(mat_vec_product(A, x))
    g = A.T @ (act - b01) / n
    return g if l2 == 0 else g + l2 * x


def hessian_weights(A, x):
    """s (1 - s), s = expit(Ax) (loss.py:295-297)."""
    a = scipy.special.expit(mat_vec_product(A, x))
    return a * (1 - a)


def hess_vec_prod(A, x, v, l2=0.0):
    """A^T (w * A v) / n + l2 v (loss.py:289-302, grad_dif=False)."""
    return hvp_from_weights(A, hessian_weights(A, x), v, l2)


def hvp_from_weights(A, w, v, l2=0.0):
    n = A.shape[0]
    Av = A @ v
    return A.T @ np.multiply(w, Av) / n + l2 * v


# ---------------------------------------------------------- cubic.py
def lanczos(op, v, m=10):
    """Three-term Lanczos, reference quirks included (cubic.py:77-111):
    absolute breakdown |beta| < 1e-6, truncation only when j < m-2, final
    alphas[-1] = v . op(v).  Returns (V d x m_eff, alphas, betas, beta)."""
    beta = 0
    v_pre = np.zeros_like(v)
    v = v / np.linalg.norm(v)
    V = np.zeros((len(v), m))
    V[:, 0] = v
    alphas = np.zeros(m)
    betas = np.zeros(m - 1)
    j = 0
    for j in range(m - 1):
        w = op(v) - beta * v_pre
        alpha = np.dot(v, w)
        alphas[j] = alpha
        w = w - alpha * v
        beta = np.linalg.norm(w)
        if np.abs(beta) < 1e-6:
            break
        betas[j] = beta
        v_pre = v
        v = w / beta
        V[:, j + 1] = v
    if m > 1 and j < m - 2:
        V = V[:, :j + 1]
        alphas = alphas[:j + 1]
        betas = betas[:j]
    alphas[-1] = np.dot(v, op(v))
    return V, alphas, betas, beta


def lanczos_cgs2(op, v, m=10, tol=1e-6):
    """Build-only extension (NOT in the reference): the same recurrence with
    classical Gram-Schmidt applied twice against every previous basis vector
    after w -= alpha v and before beta = ||w||.  Defines what
    krcn_lanczos(reorth=1) computes."""
    beta = 0
    v_pre = np.zeros_like(v)
    v = v / np.linalg.norm(v)
    V = np.zeros((len(v), m))
    V[:, 0] = v
    alphas = np.zeros(m)
    betas = np.zeros(m - 1)
    j = 0
    for j in range(m - 1):
        w = op(v) - beta * v_pre
        alpha = np.dot(v, w)
        alphas[j] = alpha
        w = w - alpha * v
        for _ in range(2):
            Vk = V[:, :j + 1]
            w = w - Vk @ (Vk.T @ w)
        beta = np.linalg.norm(w)
        if np.abs(beta) < tol:
            break
        betas[j] = beta
        v_pre = v
        v = w / beta
        V[:, j + 1] = v
    if m > 1 and j < m - 2:
        V = V[:, :j + 1]
        alphas = alphas[:j + 1]
        betas = betas[:j]
    alphas[-1] = np.dot(v, op(v))
    return V, alphas, betas, beta


def cubic_solver_root(g, H, M, it_max=100, epsilon=1e-8, r0=0.1):
    """Newton on lam^2 - M^2 ||s(lam)||^2 for min <g,s> + 1/2 s^T H s + M/3 ||s||^3
    (cubic.py:40-75, dense branch)."""
    eye = np.eye(len(g))

    def lp_solve(Am, rhs):
        return solve(Am, rhs, assume_a="pos")

    def func(lam):
        s_lam = -lp_solve(H + lam * eye, g)
        return lam ** 2 - M ** 2 * np.linalg.norm(s_lam) ** 2

    def grad(lam):
        s_lam = -lp_solve(H + lam * eye, g)
        d = -2 * np.dot(s_lam, lp_solve(H + lam * eye, s_lam))
        return 2 * lam - M ** 2 * d

    sol = root_scalar(func, fprime=grad, x0=r0, method="newton", maxiter=it_max, xtol=epsilon)
    r = sol.root
    s = -lp_solve(H + r * eye, g)
    ns = la.norm(s)
    dec = r / 2 * ns ** 2 - M / 3 * ns ** 3 - np.dot(g, s) / 2
    return s, sol.iterations, r, dec


def krylov_crn(A, b, x0, m=10, reg_coef=1e-3, it_max=10, beta=0.5, solver_eps=1e-8, l2=0.0,
               lanczos_fn=lanczos):
    """`it_max` steps of Cubic_Krylov_LS.step (cubic.py:265-309) from x0.
    Returns a dict of per-step arrays: value (after the step), reg_coef, r0,
    solver_it (cumulative), m_eff, and the iterates xs (x0 first)."""
    b01 = labels01(b)
    x = np.array(x0, dtype=np.float64, copy=True)
    fval = value(A, b01, x, l2)
    out = {"value": [], "reg_coef": [], "r0": [], "solver_it": [], "m_eff": [], "xs": [x.copy()]}
    r0 = 0.1
    solver_it = 0
    for _ in range(it_max):
        g = gradient(A, b01, x, l2)
        w = hessian_weights(A, x)
        V, alphas, betas, _ = lanczos_fn(lambda v: hvp_from_weights(A, w, v, l2), g, m)
        T = np.diag(alphas) + np.diag(betas, -1) + np.diag(betas, 1)
        e1 = np.zeros(len(alphas))
        e1[0] = 1
        gs = np.linalg.norm(g) * e1
        rc = reg_coef * beta
        s, its, r0_new, dec = cubic_solver_root(gs, T, rc, epsilon=solver_eps, r0=r0)
        x_new = x + V @ s
        f_new = value(A, b01, x_new, l2)
        k = 0
        while f_new > fval - dec and k < 20:
            rc = rc / beta
            s, its, r0_new, dec = cubic_solver_root(gs, T, rc, epsilon=solver_eps, r0=r0)
            x_new = x + V @ s
            f_new = value(A, b01, x_new, l2)
            k += 1
        x, reg_coef, fval, r0 = x_new, rc, f_new, r0_new
        solver_it += its
        out["value"].append(fval)
        out["reg_coef"].append(reg_coef)
        out["r0"].append(r0)
        out["solver_it"].append(solver_it)
        out["m_eff"].append(len(alphas))
        out["xs"].append(x.copy())
    return {k: np.asarray(v) for k, v in out.items()}
