"""HIP objective kernels vs the reference's golden vectors and the oracle.

Tolerances (fp64): rel 1e-13 (max-norm) for Ax, weights, gradient and the
HVP — the HIP path sums rows in a different (fixed) order than scipy; the
measured gap is ~1e-16.  With the sequential lane policy the HVP is
bit-identical to scipy's csr_matvec/csc_matvec given the same weights.
fp32: rel 1e-5 against the fp64 reference.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import krcn
import krcn_oracle as O
from conftest import golden_csr, load_golden, rel_err
from krcn import synth

pytestmark = pytest.mark.gpu

DEV = "cuda"
LANES = [0, 1, 2, 4, 8, 16, 32, 64]


def t(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def h(x):
    torch.cuda.synchronize()
    return x.cpu().numpy()


@pytest.mark.parametrize("lanes", LANES)
def test_hvp_gradient_value_vs_golden(f1, lanes):
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A, lanes=(lanes, lanes))
    b01 = t(O.labels01(f1["b"]))
    for i in range(2):
        x = t(f1[f"x{i}"])
        Ax = X.matvec(x)
        assert rel_err(h(Ax), f1[f"Ax{i}"]) < 1e-13
        w = X.weights(Ax)
        assert rel_err(h(w), O.hessian_weights(A, f1[f"x{i}"])) < 1e-13
        assert rel_err(h(X.gradient(Ax, b01)), f1[f"grad{i}"]) < 1e-13
        assert rel_err(h(X.gradient(Ax, b01, x, l2=0.01)), f1[f"grad{i}_l2"]) < 1e-13
        assert abs(X.loss_mean(Ax, b01) - f1[f"value{i}"]) < 1e-13 * abs(f1[f"value{i}"])
        for k in range(3):
            y = X.hvp(w, t(f1[f"v{k}"]))
            assert rel_err(h(y), f1[f"hvp{i}_{k}"]) < 1e-13
        y = X.hvp(w, t(f1["v0"]), l2=0.01)
        assert rel_err(h(y), f1[f"hvp{i}_0_l2"]) < 1e-13


def test_sequential_policy_is_bitwise_scipy(f1):
    """1 lane per row, left-to-right sums, no FMA: the order of scipy's loops."""
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A, lanes=(1, 1))
    w_host = O.hessian_weights(A, f1["x1"])
    for k in range(3):
        v = f1[f"v{k}"]
        y = h(X.hvp(t(w_host), t(v)))
        np.testing.assert_array_equal(y, O.hvp_from_weights(A, w_host, v))
        np.testing.assert_array_equal(h(X.matvec(t(v))), A @ v)


@pytest.mark.parametrize("cfg,skew", [("rcv1", False), ("news20", True)])
def test_sequential_policy_bitwise_on_real_shapes(cfg, skew):
    """lanes = (1, 1) with the AUTO format on data whose X^T has rows over 32
    elements (rcv1: up to ~60; the skewed news20 shape: thousands): the auto
    policy may still pick jagged plans, but never their long-row wave sums or
    slice groups, so rmatvec and the HVP stay scipy's csc_matvec bit for bit
    (include/krcn.h, KRCN_LANES_SEQUENTIAL)."""
    A, _ = synth.make_problem(cfg, skew=skew, n=4000 if skew else None, d=60_000 if skew else None,
                              nnz=400_000 if skew else None)
    X = krcn.DeviceCSR(A, lanes=(1, 1))
    rng = np.random.default_rng(7)
    u = rng.standard_normal(A.shape[0])
    v = rng.standard_normal(A.shape[1])
    w = rng.uniform(0.01, 0.25, A.shape[0])
    np.testing.assert_array_equal(h(X.rmatvec(t(u))), (A.T @ u) / A.shape[0])
    np.testing.assert_array_equal(h(X.matvec(t(v))), A @ v)
    np.testing.assert_array_equal(h(X.hvp(t(w), t(v))), O.hvp_from_weights(A, w, v))


def test_l2_zero_hvp_signed_zeros():
    """krcn_hvp with l2 == 0 stores X^T(..)/n without the reference's + 0 * v
    (include/krcn.h).  The two agree bit for bit, the sign of zero included,
    because a row sum of X^T is never -0: it starts from +0, and +0 + (-0)
    and x + (-x) both round to +0.  Columns that make s = 0 three ways (empty;
    one product -1 * (+0) = -0; two products that cancel exactly) against v
    entries that are negative, -0 and +0: the uint64 patterns of y equal the
    oracle's A.T @ u / n + 0 * v (sequential lanes: scipy's order)."""
    rows = [0, 1, 2, 2, 3, 3]
    cols = [1, 2, 3, 3 + 1, 5, 3 + 1]
    vals = [-1.0, 2.0, 1.5, -1.5, 0.25, 1.5]
    # row 0: col 1 (u_0 = w_0 * (-1 * v_1) with v_1 = -0 -> u_0 = +0, X^T col 1: -1 * (+0) = -0)
    # row 2: cols 3, 4 with equal and opposite products into col ... (cancellation below)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(4, 8))
    A.sum_duplicates()
    A.sort_indices()
    X = krcn.DeviceCSR(A, lanes=(1, 1))
    w = np.array([0.25, 0.2, 0.125, 0.1])
    for v in (np.array([-3.0, -0.0, 1.0, -2.0, -2.0, 0.5, -1.0, -0.0]),
              np.array([0.0, -0.0, -1.0, 4.0, 4.0, -0.0, -5.0, 0.0])):
        y = h(X.hvp(t(w), t(v)))
        ref = O.hvp_from_weights(A, w, v)
        np.testing.assert_array_equal(y.view(np.uint64), ref.view(np.uint64))
        assert not np.signbit(y[[0, 6, 7]]).any()   # empty columns: +0 whatever the sign of v
    # exact cancellation inside one column: u = (1, -1) on two rows of equal values
    B = sp.csr_matrix((np.array([3.0, 3.0]), (np.array([0, 1]), np.array([0, 0]))), shape=(2, 2))
    XB = krcn.DeviceCSR(B, lanes=(1, 1))
    yb = h(XB.rmatvec(t(np.array([1.0, -1.0]))))
    np.testing.assert_array_equal(yb.view(np.uint64), ((B.T @ np.array([1.0, -1.0])) / 2).view(np.uint64))
    assert not np.signbit(yb).any()


def test_reserved_lanczos_allocates_nothing():
    """After krcn_csr_reserve(m, reorth) the recurrence owns no new device
    memory: Lanczos calls up to m, with and without CGS2, leave the handle's
    owned bytes unchanged (include/krcn.h: krcn_lanczos allocates nothing)."""
    A, _ = synth.make_problem("rcv1")
    X = krcn.DeviceCSR(A)
    X.reserve(50, reorth=True)
    before = X.owned_bytes()
    w = t(np.full(A.shape[0], 0.2))
    g = t(np.random.default_rng(3).standard_normal(A.shape[1]))
    for m, ro in ((10, False), (50, False), (50, True), (20, True)):
        X.lanczos(w, g, m, reorth=ro)
    assert X.owned_bytes() == before


def test_transpose_is_stable_csc(f1):
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A)
    colptr, rowidx, vals = X.transpose_arrays()
    C = A.tocsc()
    np.testing.assert_array_equal(h(colptr), C.indptr)
    np.testing.assert_array_equal(h(rowidx), C.indices)
    np.testing.assert_array_equal(h(vals), C.data)


@pytest.mark.parametrize("shape,nnz", [((1, 1), 1), ((1, 7), 5), ((9, 1), 4), ((5, 6), 0), ((300, 40), 3000)])
def test_edge_shapes(shape, nnz):
    rng = np.random.default_rng(nnz)
    n, d = shape
    dense = np.zeros(shape)
    if nnz:
        flat = rng.choice(n * d, size=min(nnz, n * d), replace=False)
        dense.flat[flat] = rng.uniform(-1, 1, size=len(flat))
    A = sp.csr_matrix(dense)
    x = rng.uniform(-1, 1, size=d)
    v = rng.standard_normal(d)
    X = krcn.DeviceCSR(A)
    Ax = X.matvec(t(x))
    np.testing.assert_allclose(h(Ax), A @ x, rtol=1e-14, atol=1e-15)
    w = X.weights(Ax)
    y = X.hvp(w, t(v))
    np.testing.assert_allclose(h(y), O.hess_vec_prod(A, x, v), rtol=1e-13, atol=1e-16)


def test_fp32_hvp(f1):
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A, dtype=torch.float32)
    x = f1["x1"]
    w = X.weights(X.matvec(t(x, torch.float32)))
    for k in range(3):
        y = X.hvp(w, t(f1[f"v{k}"], torch.float32))
        assert rel_err(h(y), f1[f"hvp1_{k}"]) < 1e-5


def test_hvp_properties_and_determinism():
    """Size-independent properties on a news20-scale-per-row problem:
    symmetry <u,Hv> = <Hu,v>, PSD <v,Hv> >= 0, linearity, and bitwise
    run-to-run reproducibility (no atomics anywhere)."""
    A, b = synth.make_problem(None, seed=3, n=4000, d=200_000, nnz=1_800_000)
    X = krcn.DeviceCSR(A)
    x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=DEV)
    w = X.weights(X.matvec(x))
    g = torch.Generator(device="cpu").manual_seed(0)
    u = torch.randn(A.shape[1], generator=g, dtype=torch.float64).to(DEV)
    v = torch.randn(A.shape[1], generator=g, dtype=torch.float64).to(DEV)
    Hu, Hv = X.hvp(w, u), X.hvp(w, v)
    s1, s2 = X.dot(u, Hv), X.dot(Hu, v)
    assert abs(s1 - s2) <= 1e-12 * abs(s1)
    assert X.dot(v, Hv) >= 0
    Hlin = X.hvp(w, (2.0 * u + 3.0 * v).contiguous())
    assert rel_err(h(Hlin), h(2.0 * Hu + 3.0 * Hv)) < 1e-13
    np.testing.assert_array_equal(h(X.hvp(w, v)), h(Hv))


@pytest.mark.parametrize("cfg", ["rcv1", "news20"])
def test_fullshape_vs_golden_statistics(cfg):
    f = load_golden(f"f5_{cfg}.npz")
    A, b = synth.make_problem(cfg)
    X = krcn.DeviceCSR(A)
    b01 = t(O.labels01(b))
    x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=DEV)
    Ax = X.matvec(x)
    val = X.loss_mean(Ax, b01)
    assert abs(val - f["value"]) <= 1e-13 * abs(f["value"])
    g = X.gradient(Ax, b01)
    st = int(f["stride"])
    assert rel_err(h(g)[::st], f["g_sample"]) < 1e-13
    gn = X.diff_norm(g)
    assert abs(gn - f["g_norm"]) <= 1e-13 * f["g_norm"]
    w = X.weights(Ax)
    y = X.hvp(w, (g / gn).contiguous())
    assert rel_err(h(y)[::st], f["y_sample"]) < 1e-12
    assert abs(X.diff_norm(y) - f["y_norm"]) <= 1e-12 * f["y_norm"]
