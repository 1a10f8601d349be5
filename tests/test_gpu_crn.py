"""End-to-end: the drop-in Cubic_Krylov_LS (device HVP/Lanczos, host cubic
subproblem) reproduces the reference's Krylov-CRN trajectory.

Tolerance: x_k and f_k within 1e-10 relative over 10 steps;
the line-search decisions (reg_coef, solver iteration counts) must be equal.
"""
import numpy as np
import pytest

from conftest import load_golden, rel_err
from krcn import synth
from optimizer.cubic import Cubic_Krylov_LS, Lanczos
from optimizer.loss import LogisticRegression

pytestmark = pytest.mark.gpu


def test_trajectory_10_steps(f4):
    n, d, nnz = (int(v) for v in f4["shape"])
    A, b = synth.make_problem(None, seed=int(f4["seed"]), n=n, d=d, nnz=nnz)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="krylov", subspace_dim=10, tolerance=1e-9,
                          tqdm=False)
    tr = opt.run(x0=np.full(d, 0.5), it_max=10)
    opt.compute_loss_of_iterates()
    xs = np.asarray(tr.xs)
    assert xs.shape == f4["xs"].shape
    assert rel_err(xs, f4["xs"]) < 1e-10
    assert tr.its == list(f4["its"])
    assert tr.solver_its == list(f4["solver_its"])
    np.testing.assert_allclose(tr.loss_vals, f4["loss_vals"], rtol=1e-10)
    assert opt.reg_coef == f4["final_reg_coef"]
    assert abs(opt.value - f4["final_value"]) <= 1e-10 * abs(f4["final_value"])


def test_rcv1_three_steps():
    f = load_golden("f5_rcv1.npz")
    A, b = synth.make_problem("rcv1")
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=int(f["m"]), tolerance=1e-9,
                          tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=3)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, f["crn_loss_vals"], rtol=1e-10)
    x = opt.x.cpu().numpy()
    st = int(f["stride"])
    assert rel_err(x[::st], f["crn_final_x_sample"]) < 1e-10


def test_numpy_api_and_lanczos_wrapper(f1):
    from conftest import golden_csr
    A = golden_csr(f1)
    loss = LogisticRegression(A, f1["b"], l1=0, l2=0, store_mat_vec_prod=True)
    x = f1["x0"]
    assert rel_err(loss.mat_vec_product(x), f1["Ax0"]) < 1e-13
    assert abs(loss.value(x) - f1["value0"]) <= 1e-13 * abs(f1["value0"])
    g = loss.gradient(x)
    assert isinstance(g, np.ndarray) and rel_err(g, f1["grad0"]) < 1e-13
    assert rel_err(loss.hess_vec_prod(x, f1["v1"]), f1["hvp0_1"]) < 1e-13
    V, al, be, beta = Lanczos(loss.hess_operator(x), g, m=10)
    f2 = load_golden("f2_lanczos.npz")
    assert V.shape == (A.shape[1], 10)
    assert rel_err(al, f2["alphas_m10"]) < 1e-11
    assert loss.f_opt == loss.value(x)


def test_async_checkpoints_hold_each_iterate(f4):
    """Trace checkpoints are async D2H copies into pinned memory
    (loss.to_host_async): every stored iterate is its own buffer, the last one
    equals the final device iterate once run() returns, and each equals a
    synchronous copy of the same trajectory (the golden xs in
    test_trajectory_10_steps pin the values)."""
    n, d, nnz = (int(v) for v in f4["shape"])
    A, b = synth.make_problem(None, seed=int(f4["seed"]), n=n, d=d, nnz=nnz)
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="krylov", subspace_dim=10, tolerance=1e-9,
                          tqdm=False)
    tr = opt.run(x0=np.full(d, 0.5), it_max=6)
    np.testing.assert_array_equal(tr.xs[-1], opt.x.cpu().numpy())
    assert len({x.__array_interface__["data"][0] for x in tr.xs}) == len(tr.xs)
    loss2 = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    loss2.to_host_async = loss2.to_host   # synchronous copies
    opt2 = Cubic_Krylov_LS(loss=loss2, reg_coef=1e-3, label="krylov", subspace_dim=10, tolerance=1e-9,
                           tqdm=False)
    tr2 = opt2.run(x0=np.full(d, 0.5), it_max=6)
    np.testing.assert_array_equal(np.asarray(tr.xs), np.asarray(tr2.xs))
