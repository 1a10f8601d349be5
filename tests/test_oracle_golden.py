"""Pin the CPU oracle (oracle/krcn_oracle.py) to the reference's own outputs.

The golden vectors were produced by importing the reference
(tests/golden/make_golden.py).  The oracle makes the same scipy/numpy calls,
so agreement is bitwise except where noted.
"""
import hashlib

import numpy as np
import pytest

import krcn_oracle as O
from conftest import golden_csr, load_golden, rel_err
from krcn import synth


def test_hvp_value_gradient_bitwise(f1):
    A = golden_csr(f1)
    b01 = O.labels01(f1["b"])
    for i in range(2):
        x = f1[f"x{i}"]
        np.testing.assert_array_equal(O.mat_vec_product(A, x), f1[f"Ax{i}"])
        assert O.value(A, b01, x) == f1[f"value{i}"]
        np.testing.assert_array_equal(O.gradient(A, b01, x), f1[f"grad{i}"])
        for k in range(3):
            np.testing.assert_array_equal(O.hess_vec_prod(A, x, f1[f"v{k}"]), f1[f"hvp{i}_{k}"])
        np.testing.assert_array_equal(O.gradient(A, b01, x, l2=0.01), f1[f"grad{i}_l2"])
        np.testing.assert_array_equal(O.hess_vec_prod(A, x, f1["v0"], l2=0.01), f1[f"hvp{i}_0_l2"])
        assert O.value(A, b01, x, l2=0.01) == f1[f"value{i}_l2"]


def test_lanczos_bitwise(f1, f2):
    A = golden_csr(f1)
    x = f1["x0"]
    w = O.hessian_weights(A, x)
    op = lambda v: O.hvp_from_weights(A, w, v)  # noqa: E731
    for m in (1, 10, 50):
        V, al, be, beta = O.lanczos(op, f2["g"], m)
        np.testing.assert_array_equal(al, f2[f"alphas_m{m}"])
        np.testing.assert_array_equal(be, f2[f"betas_m{m}"])
        np.testing.assert_array_equal(V, f2[f"V_m{m}"])
        assert beta == f2[f"beta_m{m}"]


@pytest.mark.parametrize("r,ms", [(1, (2, 3, 5)), (3, (4, 5, 10))])
def test_lanczos_breakdown_quirks(f2, r, ms):
    A = golden_csr(f2, f"r{r}_")
    b01 = O.labels01(f2[f"r{r}_b"])
    x = np.full(A.shape[1], 0.5)
    g = O.gradient(A, b01, x)
    np.testing.assert_array_equal(g, f2[f"r{r}_g"])
    w = O.hessian_weights(A, x)
    for m in ms:
        V, al, be, beta = O.lanczos(lambda v: O.hvp_from_weights(A, w, v), g, m)
        key = f"r{r}_m{m}"
        assert V.shape == f2[f"{key}_V"].shape
        np.testing.assert_array_equal(al, f2[f"{key}_alphas"])
        np.testing.assert_array_equal(be, f2[f"{key}_betas"])
        np.testing.assert_array_equal(V, f2[f"{key}_V"])
        # the quirk: breakdown at j == m-2 keeps a zero last column and betas[-1] == 0
        if m == r + 1:
            assert np.all(V[:, -1] == 0) and be[-1] == 0


def test_cubic_solver_root_bitwise(f3):
    for m in (3, 10, 50):
        for k in range(3):
            key = f"m{m}_k{k}"
            s, its, r, dec = O.cubic_solver_root(f3[f"{key}_g"], f3[f"{key}_T"], float(f3[f"{key}_M"]),
                                                 epsilon=1e-8, r0=float(f3[f"{key}_r0"]))
            np.testing.assert_array_equal(s, f3[f"{key}_s"])
            assert its == f3[f"{key}_its"] and r == f3[f"{key}_r"] and dec == f3[f"{key}_dec"]


def test_krylov_crn_trajectory(f4):
    n, d, nnz = (int(v) for v in f4["shape"])
    A, b = synth.make_problem(None, seed=int(f4["seed"]), n=n, d=d, nnz=nnz)
    out = O.krylov_crn(A, b, np.full(d, 0.5), m=10, reg_coef=1e-3, it_max=10)
    np.testing.assert_allclose(out["xs"], f4["xs"], rtol=0, atol=1e-13)
    assert out["solver_it"][-1] == f4["solver_its"][-1]
    np.testing.assert_allclose(out["value"][-1], f4["final_value"], rtol=1e-14)
    np.testing.assert_allclose(out["reg_coef"][-1], f4["final_reg_coef"], rtol=0)


@pytest.mark.parametrize("cfg,m", [("rcv1", 50), ("news20", 10)])
def test_fullshape_statistics(cfg, m):
    f = load_golden(f"f5_{cfg}.npz")
    A, b = synth.make_problem(cfg)
    assert A.nnz == int(f["nnz"])
    b01 = O.labels01(b)
    x = np.full(A.shape[1], 0.5)
    assert O.value(A, b01, x) == f["value"]
    g = O.gradient(A, b01, x)
    st = int(f["stride"])
    np.testing.assert_array_equal(g[::st], f["g_sample"])
    w = O.hessian_weights(A, x)
    y = O.hvp_from_weights(A, w, g / np.linalg.norm(g))
    np.testing.assert_array_equal(y[::st], f["y_sample"])
    _, al, be, _ = O.lanczos(lambda v: O.hvp_from_weights(A, w, v), g, m)
    # alphas[:m-1] and betas are prefixes of the golden m-step run
    assert rel_err(al[:m - 1], f["alphas"][:m - 1]) == 0.0
    assert rel_err(be, f["betas"][:m - 1]) == 0.0


def test_synth_generator_is_stable():
    """The GPU box regenerates inputs from (config, seed); pin the bytes."""
    A, b = synth.make_problem(None, seed=5, n=300, d=1000, nnz=4000)
    h = hashlib.sha256()
    for arr in (A.indptr, A.indices, A.data, b):
        h.update(np.ascontiguousarray(arr).tobytes())
    assert h.hexdigest() == SYNTH_HASH


SYNTH_HASH = "ec9a7568eaf1ec3bcebe9e4c3f49394bfe6b1e31378c4ba4ac5e24894ff5173d"
