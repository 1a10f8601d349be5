"""Execution-plan coverage: both tile formats (wave tiles, and block tiles
stored sorted by gather index), every lane width, forced column slicing (the
XCD-sliced path normally only triggers on news20-sized vectors) and the
long-row path (rows longer than a tile's 512 / 2048 nonzeros), on matrices
with empty rows/columns.  Reference: the oracle (scipy), fp64.

Bitwise claims: with 1 lane per row and no slicing the kernels sum in
scipy's order, so Ax / HVP equal csr_matvec / csc_matvec exactly, long rows
included.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import krcn
import krcn_oracle as O
from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, torch.float64)


def long_row_matrix(seed=0):
    """Row lengths 0..12 plus rows of 513, 600, 1500 and 5000 nonzeros; every
    9th row and a band of columns empty; column counts skewed (a few columns
    are hit by most rows, as in real text data)."""
    rng = np.random.default_rng(seed)
    n, d = 3000, 9000
    lengths = rng.integers(0, 13, size=n)
    lengths[::9] = 0
    for r, L in ((17, 513), (18, 600), (400, 1500), (2999, 5000), (1000, 511), (1001, 509)):
        lengths[r] = L
    live = np.setdiff1d(np.arange(d), np.arange(4000, 4100))
    hot = live[:40]
    rows, cols = [], []
    for i, L in enumerate(lengths):
        if L == 0:
            continue
        k_hot = min(L // 3, len(hot))
        c = np.concatenate([rng.choice(hot, size=k_hot, replace=False),
                            rng.choice(np.setdiff1d(live, hot), size=L - k_hot, replace=False)])
        c = np.sort(c)
        rows.append(np.full(len(c), i))
        cols.append(c)
    A = sp.csr_matrix((rng.uniform(-1, 1, size=sum(map(len, cols))),
                       (np.concatenate(rows), np.concatenate(cols))), shape=(n, d))
    A.sort_indices()
    b = np.where(rng.uniform(size=n) < 0.5, -1.0, 1.0)
    return A, b


@pytest.fixture(scope="module")
def problem():
    A, b = long_row_matrix()
    x = np.random.default_rng(1).uniform(-0.2, 0.2, size=A.shape[1])
    v = np.random.default_rng(2).standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    return A, b, x, v, w


@pytest.mark.parametrize("slicing", [1, 8, 16])
@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 16, 32, 64])
def test_plans_match_oracle(problem, slicing, lanes):
    A, b, x, v, w = problem
    X = krcn.DeviceCSR(A, lanes=(lanes, lanes), slicing=slicing, fmt=krcn.KRCN_FORMAT_WAVE)
    info = X.plan_info()
    assert info["pass1"][0] == (1 if slicing == 1 or lanes == 1 else slicing)
    Ax = X.matvec(t(x))
    assert rel_err(Ax.cpu().numpy(), A @ x) < 1e-13
    y = X.hvp(t(w), t(v))
    yr = O.hvp_from_weights(A, w, v)
    assert rel_err(y.cpu().numpy(), yr) < 1e-13
    g = X.gradient(Ax, t(O.labels01(b)))
    assert rel_err(g.cpu().numpy(), O.gradient(A, O.labels01(b), x)) < 1e-13
    if lanes == 1:      # sequential policy never slices: scipy order, bit for bit
        np.testing.assert_array_equal(y.cpu().numpy(), yr)
        np.testing.assert_array_equal(Ax.cpu().numpy(), A @ x)


@pytest.mark.parametrize("slicing", [1, 8, 16])
@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 16, 32, 64])
def test_sorted_tiles_match_oracle(problem, slicing, lanes):
    A, b, x, v, w = problem
    X = krcn.DeviceCSR(A, lanes=(lanes, lanes), slicing=slicing, fmt=krcn.KRCN_FORMAT_SORTED)
    info = X.plan_info()
    assert info["pass1"][0] == -(1 if slicing == 1 or lanes == 1 else slicing)
    assert info["pass2"][0] < 0
    Ax = X.matvec(t(x))
    assert rel_err(Ax.cpu().numpy(), A @ x) < 1e-13
    y = X.hvp(t(w), t(v))
    yr = O.hvp_from_weights(A, w, v)
    assert rel_err(y.cpu().numpy(), yr) < 1e-13
    g = X.gradient(Ax, t(O.labels01(b)))
    assert rel_err(g.cpu().numpy(), O.gradient(A, O.labels01(b), x)) < 1e-13
    if lanes == 1:      # products return to CSR slots before the row sums: scipy order
        np.testing.assert_array_equal(y.cpu().numpy(), yr)
        np.testing.assert_array_equal(Ax.cpu().numpy(), A @ x)


@pytest.mark.parametrize("lanes", [2, 8, 32])
def test_sorted_equals_wave_bitwise(problem, lanes):
    """Same lanes, no slicing: the sorted format only reorders the loads; each
    row's products go back to their CSR slots and lane q sums the elements
    with (offset in row) % L == q in both formats, long rows included (sort
    segments are multiples of L) -> bit-identical results."""
    A, b, x, v, w = problem
    Xw = krcn.DeviceCSR(A, lanes=(lanes, lanes), slicing=1, fmt=krcn.KRCN_FORMAT_WAVE)
    Xs = krcn.DeviceCSR(A, lanes=(lanes, lanes), slicing=1, fmt=krcn.KRCN_FORMAT_SORTED)
    np.testing.assert_array_equal(Xw.matvec(t(x)).cpu().numpy(), Xs.matvec(t(x)).cpu().numpy())
    np.testing.assert_array_equal(Xw.hvp(t(w), t(v)).cpu().numpy(), Xs.hvp(t(w), t(v)).cpu().numpy())


def test_sorted_tiles_skewed_synth():
    """rcv1-shaped skewed matrix (power-law columns, lognormal rows) through the
    automatic format choice and both forced formats."""
    from krcn import synth
    A, b = synth.make_problem("rcv1", skew=True, n=6000, nnz=400_000)
    x = np.random.default_rng(3).uniform(-0.3, 0.3, size=A.shape[1])
    v = np.random.default_rng(4).standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    yr = O.hvp_from_weights(A, w, v)
    for fmt in (krcn.KRCN_FORMAT_AUTO, krcn.KRCN_FORMAT_WAVE, krcn.KRCN_FORMAT_SORTED):
        X = krcn.DeviceCSR(A, fmt=fmt)
        assert rel_err(X.hvp(t(w), t(v)).cpu().numpy(), yr) < 1e-13
        assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13


@pytest.mark.parametrize("fmt", [1, 2])
@pytest.mark.parametrize("slicing", [0, 8])
def test_lanczos_with_slices(problem, slicing, fmt):
    A, b, x, v, w = problem
    X = krcn.DeviceCSR(A, slicing=slicing, fmt=fmt)
    g = X.gradient(X.matvec(t(x)), t(O.labels01(b)))
    V, al, be, info = X.lanczos(t(w), g, 12)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.cpu().numpy(), 12)
    assert info.m_eff == 12
    # this skewed operator amplifies rounding: a 1e-16 HVP perturbation moves
    # the oracle's alphas by ~1e-11 at m = 12 (measured), hence 1e-9
    assert rel_err(al, al_r) < 1e-9
    assert rel_err(be, be_r) < 1e-9


def test_sliced_equals_unsliced_within_rounding(problem):
    A, b, x, v, w = problem
    y0 = krcn.DeviceCSR(A, slicing=1).hvp(t(w), t(v)).cpu().numpy()
    y8 = krcn.DeviceCSR(A, slicing=8).hvp(t(w), t(v)).cpu().numpy()
    assert rel_err(y8, y0) < 1e-14
