"""The rest of cubic_newton.py on the device kernels: Lanczos over a plain
callable, the full-space CRN (Cubic_LS "full" and "CG"), SSCN, and the
smoothness / Hessian-Lipschitz constants behind reg_coef=None — against
fixtures the reference produced (tests/golden/f2_lanczos.npz, f6_methods.npz).

Tolerances: fp64 alphas / betas 1e-11, V 1e-6 (f1's operator amplifies a 1e-16
HVP perturbation to 8e-9 in V[:, 9]); trajectories x_k / f_k 1e-10 with equal
line-search decisions where the arithmetic is the reference's up to summation
order; smoothness 1e-10 (the reference's svds vs the device Lanczos top Ritz
value).  Cubic_LS "CG" is "parity unpinned": the reference's cg(..., tol=)
raises on this scipy (cubic.py:161), so the CG-CRN is checked against the
full-space solve of the same step with the CG tolerance (rtol 1e-8) in mind.
"""
import numpy as np
import pytest
import torch

import krcn
import krcn_oracle as O
from conftest import golden_csr, load_golden, rel_err
from krcn import synth
from optimizer.cubic import SSCN, Cubic_Krylov_LS, Cubic_LS, Lanczos
from optimizer.loss import LogisticRegression

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def f6():
    return load_golden("f6_methods.npz")


def f6_problem(f6):
    n, d, nnz = (int(v) for v in f6["shape"])
    return synth.make_problem(None, seed=int(f6["seed"]), n=n, d=d, nnz=nnz)


# ------------------------------------------------------------ Lanczos(callable)
@pytest.mark.parametrize("m", [1, 10])
def test_lanczos_numpy_callable_vs_golden(f1, f2, m):
    A = golden_csr(f1)
    loss = LogisticRegression(A, f1["b"], l1=0, l2=0, store_mat_vec_prod=True)
    x = f1["x0"]
    g = loss.gradient(x)
    V, al, be, beta = Lanczos(lambda v: loss.hess_vec_prod(x, v), g, m=m)
    assert isinstance(V, np.ndarray) and V.shape == f2[f"V_m{m}"].shape
    assert rel_err(al, f2[f"alphas_m{m}"]) < 1e-11
    assert rel_err(be, f2[f"betas_m{m}"]) < 1e-11
    assert np.abs(V - f2[f"V_m{m}"]).max() < 1e-6
    assert abs(beta - float(f2[f"beta_m{m}"])) <= 1e-11 * max(abs(float(f2[f"beta_m{m}"])), 1e-300)


def test_lanczos_device_callable_vs_golden(f1, f2):
    A = golden_csr(f1)
    loss = LogisticRegression(A, f1["b"], l1=0, l2=0, store_mat_vec_prod=True)
    x = loss.to_device(f1["x0"])
    g = loss.gradient(x)
    V, al, be, _ = Lanczos(lambda v: loss.hess_vec_prod(x, v), g, m=10)
    assert isinstance(V, torch.Tensor) and V.device.type == "cuda"
    assert rel_err(al, f2["alphas_m10"]) < 1e-11
    assert rel_err(be, f2["betas_m10"]) < 1e-11
    assert np.abs(V.cpu().numpy() - f2["V_m10"]).max() < 1e-6


@pytest.mark.parametrize("r,m", [(1, 2), (1, 3), (1, 5), (3, 4), (3, 5), (3, 10)])
def test_lanczos_callable_breakdown_quirks(f2, r, m):
    """Breakdown at j = r - 1: truncation only when j < m - 2, the zero last
    column otherwise, and the final alpha overwriting the right slot
    (cubic.py:98-109), exactly as the reference returned them."""
    A = golden_csr(f2, prefix=f"r{r}_")
    loss = LogisticRegression(A, f2[f"r{r}_b"], l1=0, l2=0, store_mat_vec_prod=True)
    x = np.full(A.shape[1], 0.5)
    V, al, be, beta = Lanczos(lambda v: loss.hess_vec_prod(x, v), f2[f"r{r}_g"], m=m)
    key = f"r{r}_m{m}"
    assert V.shape == f2[f"{key}_V"].shape
    assert al.shape == f2[f"{key}_alphas"].shape and be.shape == f2[f"{key}_betas"].shape
    assert rel_err(al, f2[f"{key}_alphas"]) < 1e-11
    if be.size:
        assert rel_err(be, f2[f"{key}_betas"]) < 1e-11
    np.testing.assert_array_equal(V == 0.0, f2[f"{key}_V"] == 0.0)
    assert np.abs(V - f2[f"{key}_V"]).max() < 1e-9
    assert abs(beta) < 1e-6


# ------------------------------------------------------------ constants
def test_smoothness_and_hessian_lipschitz(f6):
    A, b = f6_problem(f6)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    assert abs(loss.smoothness - f6["smoothness"]) <= 1e-10 * f6["smoothness"]
    assert abs(loss.hessian_lipschitz - f6["hessian_lipschitz"]) <= 1e-10 * f6["hessian_lipschitz"]
    Ar, br = synth.make_problem("rcv1")       # n, d > 20000: the Frobenius branch
    lr = LogisticRegression(Ar, br, l1=0, l2=0, store_mat_vec_prod=True)
    with pytest.warns(UserWarning):
        sm = lr.smoothness
    assert abs(sm - f6["rcv1_smoothness"]) <= 1e-13 * f6["rcv1_smoothness"]
    assert abs(lr.hessian_lipschitz - f6["rcv1_hessian_lipschitz"]) <= 1e-13 * f6["rcv1_hessian_lipschitz"]


def test_krylov_with_reg_coef_none(f6):
    A, b = f6_problem(f6)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=None, label="k", subspace_dim=10, tolerance=1e-9, tqdm=False)
    assert abs(opt.reg_coef - f6["krylov_auto_reg_coef0"]) <= 1e-10 * f6["krylov_auto_reg_coef0"]
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=3)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, f6["krylov_auto_loss_vals"], rtol=1e-8)
    assert rel_err(np.asarray(tr.xs), f6["krylov_auto_xs"]) < 1e-8
    assert tr.solver_its == list(f6["krylov_auto_solver_its"])


# ------------------------------------------------------------ full-space CRN
def test_dense_hessian_vs_scipy(f1):
    A = golden_csr(f1)
    loss = LogisticRegression(A, f1["b"], l1=0, l2=0.01, store_mat_vec_prod=True)
    x = f1["x1"]
    H = loss.hessian(x)
    w = O.hessian_weights(A, x)
    ref = (A.T.multiply(w) @ A / A.shape[0]).toarray() + 0.01 * np.eye(A.shape[1])
    assert rel_err(H, ref) < 1e-13


def test_cubic_ls_full_vs_reference(f6):
    A, b = f6_problem(f6)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_LS(loss=loss, reg_coef=1e-3, label="CRN", cubic_solver="full", tolerance=1e-8, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=3)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, f6["full_loss_vals"], rtol=1e-10)
    assert rel_err(np.asarray(tr.xs), f6["full_xs"]) < 1e-10
    assert tr.solver_its == list(f6["full_solver_its"])
    assert opt.reg_coef == f6["full_reg_coef"]


def test_cg_solve_matches_dense_solve():
    A, b = synth.make_problem(None, seed=8, n=2000, d=700, nnz=40_000)
    X = krcn.DeviceCSR(A)
    x = np.random.default_rng(1).uniform(-0.5, 0.5, size=A.shape[1])
    w = O.hessian_weights(A, x)
    rhs = np.random.default_rng(2).standard_normal(A.shape[1])
    shift = 0.05
    sol, info = X.cg_solve(torch.from_numpy(w).to(DEV), torch.from_numpy(rhs).to(DEV), shift=shift, rtol=1e-10)
    H = (A.T.multiply(w) @ A / A.shape[0]).toarray() + shift * np.eye(A.shape[1])
    ref = np.linalg.solve(H, rhs)
    assert info.converged == 1 and info.info == 0 and 0 < info.iterations < 10 * A.shape[1]
    assert info.residual_norm < 1e-10 * np.linalg.norm(rhs)
    assert rel_err(sol.cpu().numpy(), ref) < 1e-8
    # scipy's early exit: b = 0 returns x = 0 without iterating
    z, info0 = X.cg_solve(torch.from_numpy(w).to(DEV), torch.zeros(A.shape[1], dtype=torch.float64, device=DEV))
    assert info0.converged == 1 and info0.iterations == 0 and not z.abs().max().item()
    # maxiter exhausted: scipy reports info = maxiter
    _, info1 = X.cg_solve(torch.from_numpy(w).to(DEV), torch.from_numpy(rhs).to(DEV), shift=shift, rtol=1e-14,
                          maxiter=3)
    assert info1.converged == 0 and info1.info == 3 and info1.iterations == 3


def test_cubic_ls_cg_tracks_the_full_solve(f6):
    """parity unpinned (see module docstring): CG-CRN vs the reference's
    full-space trajectory on the same problem."""
    A, b = f6_problem(f6)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_LS(loss=loss, reg_coef=1e-3, label="CRN", cubic_solver="CG", tolerance=1e-8, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=3)
    opt.compute_loss_of_iterates()
    assert opt.cg_iterations > 0
    np.testing.assert_allclose(tr.loss_vals, f6["full_loss_vals"], rtol=1e-6)
    assert rel_err(np.asarray(tr.xs), f6["full_xs"]) < 1e-5


# ------------------------------------------------------------ SSCN
def test_sscn_vs_reference(f6):
    A, b = f6_problem(f6)
    loss = LogisticRegression(A.tocsc(), b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = SSCN(loss=loss, reg_coef=1e-3, label="SSCN", subspace_dim=10, tolerance=1e-9, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=6)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, f6["sscn_loss_vals"], rtol=1e-10)
    assert rel_err(np.asarray(tr.xs), f6["sscn_xs"]) < 1e-10
    # SSCN's subproblem Newton runs to xtol = machine epsilon (cubic.py:365), so
    # its iteration count sits on the last bit of lam: a 1-ulp difference in the
    # partial Hessian adds or saves one final iteration (measured: 10 vs 11)
    # while s, x and f agree to 1e-10 above
    its = np.diff(tr.solver_its)
    ref_its = np.diff(f6["sscn_solver_its"])
    assert len(its) == len(ref_its) and np.abs(its - ref_its).max() <= 1


# ------------------------------------------------------------ the driver
def test_cubic_newton_driver_sequence():
    """cubic_newton.py:56-106 with the dataset download and plotting left out:
    every optimizer it builds runs on the device path and decreases the loss."""
    A, b = synth.make_problem(None, seed=12, n=1500, d=900, nnz=20_000)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    loss_csc = LogisticRegression(A.tocsc(), b, l1=0, l2=0, store_mat_vec_prod=True)
    n, dim = A.shape
    x0 = np.ones(dim) * 0.5
    cub_krylov = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="Krylov CRN (m = 10)", subspace_dim=10,
                                 tolerance=1e-9, tqdm=False)
    cub_krylov_bench = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="Benchmark Krylov CRN (m = 20)",
                                       subspace_dim=20, tolerance=1e-9, tqdm=False)
    cubic_solver = "full" if dim < 500 else "CG"
    cub_root = Cubic_LS(loss=loss, reg_coef=1e-3, label="CRN", cubic_solver=cubic_solver, tolerance=1e-8,
                        tqdm=False)
    sscn_list = [SSCN(loss=loss_csc, reg_coef=1e-3, label=f"SSCN (m = {m})", subspace_dim=m, tolerance=1e-9,
                      tqdm=False) for m in (10,)]
    it_max, time_max = 3, 60
    cub_root.run(x0=x0, it_max=it_max, t_max=time_max)
    cub_root.compute_loss_of_iterates()
    time_max = max(cub_root.trace.ts[-1], time_max)
    for algs in sscn_list:
        algs.run(x0=x0, it_max=it_max, t_max=time_max)
        algs.compute_loss_of_iterates()
    cub_krylov.run(x0=x0, it_max=it_max, t_max=time_max)
    cub_krylov.compute_loss_of_iterates()
    cub_krylov_bench.run(x0=x0, it_max=5 * it_max, t_max=5 * time_max)
    cub_krylov_bench.compute_loss_of_iterates()
    for opt in (cub_root, *sscn_list, cub_krylov, cub_krylov_bench):
        lv = np.asarray(opt.trace.loss_vals)
        assert len(lv) >= 2 and np.all(np.diff(lv) <= 1e-12), opt.label
        assert lv[-1] < lv[0], opt.label


def test_sscn_without_stored_products(f6):
    """store_mat_vec_prod=False (the reference's default, loss.py:186): the
    cache starts as the reference's never-read zero vector; SSCN must run and
    give the stored-product trajectory (it used to raise)."""
    A, b = f6_problem(f6)
    loss = LogisticRegression(A.tocsc(), b, l1=0, l2=0, store_mat_vec_prod=False)
    opt = SSCN(loss=loss, reg_coef=1e-3, label="SSCN", subspace_dim=10, tolerance=1e-9, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=6)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, f6["sscn_loss_vals"], rtol=1e-10)
    assert rel_err(np.asarray(tr.xs), f6["sscn_xs"]) < 1e-10


def test_smoothness_mixed_sign_columns():
    """Columns of opposite sign put the constant start vector in the null space
    of X^T X (X 1 = 0): the first Lanczos breaks down at once on an invariant
    subspace, and the estimate must restart instead of returning 0.  Here
    X^T X / n = [[1, -1], [-1, 1]] (+ a small third column), so sigma_max^2 / n
    = 2 + O(1e-2) and smoothness = 0.25 sigma_max^2 / n (loss.py:308-320,
    scipy svds on the host as the check)."""
    import scipy.sparse as sp
    from scipy.sparse.linalg import svds
    n = 64
    rng = np.random.default_rng(5)
    third = rng.uniform(-0.1, 0.1, n)
    third -= third.mean()
    A = sp.csr_matrix(np.column_stack([np.ones(n), -np.ones(n), third]))
    b = np.where(rng.uniform(size=n) < 0.5, -1.0, 1.0)
    loss = LogisticRegression(A, b, l1=0, l2=0)
    sigma = svds(A, k=1, return_singular_vectors=False)[0]
    assert abs(loss.smoothness - 0.25 * sigma ** 2 / n) <= 1e-10 * 0.25 * sigma ** 2 / n


def test_cubic_ls_cg_fp32_terminates(f6):
    """fp32 device CG with the reference's rtol = 1e-8: the requested residual
    is below fp32's reach, so it is clamped to 10 ulp; every solve must
    converge well inside maxiter = 10 d (it ran to maxiter)."""
    A, b = f6_problem(f6)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True, dtype=torch.float32)
    opt = Cubic_LS(loss=loss, reg_coef=1e-3, label="CRN", cubic_solver="CG", tolerance=1e-8, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=2)
    opt.compute_loss_of_iterates()
    assert opt.cg_unconverged == 0
    assert opt.cg_iterations > 0
    np.testing.assert_allclose(tr.loss_vals, f6["full_loss_vals"][:len(tr.loss_vals)], rtol=1e-4)
