"""LDS-window format (krcn_window.hpp): the gathered vector is copied into LDS
one column slice (W = 15,872 fp64 / 31,744 fp32 entries) at a time and each
row is summed in one lane.

Coverage: both ways the format runs (accumulate: every block walks all slices
of its rows, no partials; slices: per-slice partials + combine), every tile
height (16 / 32 / 64 rows from the mean row length per slice), rows longer
than a staging chunk (256 nonzeros) up to 5000, empty rows and an empty
column band, slice ends that are not multiples of anything, fp64 and fp32,
the Lanczos recurrence through it, and the automatic choice on the
news20-shaped benchmark matrix.  Reference: the oracle (scipy).

Bitwise claim: in accumulate mode a row's running sum carries across slices
in column order, i.e. left to right over its whole CSR row, so X v and X^T u
are scipy's csr_matvec / csc_matvec bit for bit.
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
W64 = 15872


def t(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def skewed(n, d, mean_len, seed, long_rows=((17, 600), (400, 1500), (5, 257), (6, 5000))):
    """Poisson row lengths, every 9th row empty, an empty column band, some
    long rows; sorted unique columns; U(-1, 1) values."""
    rng = np.random.default_rng(seed)
    lengths = rng.poisson(mean_len, size=n)
    lengths[::9] = 0
    for r, L in long_rows:
        if r < n:
            lengths[r] = min(L, d - 200)
    live = np.setdiff1d(np.arange(d), np.arange(d // 3, d // 3 + 150))
    rows, cols = [], []
    for i, L in enumerate(lengths):
        if L == 0:
            continue
        c = np.sort(rng.choice(live, size=L, replace=False))
        rows.append(np.full(L, i))
        cols.append(c)
    A = sp.csr_matrix((rng.uniform(-1, 1, size=int(lengths.sum())),
                       (np.concatenate(rows), np.concatenate(cols))), shape=(n, d))
    A.sort_indices()
    b = np.where(rng.uniform(size=n) < 0.5, -1.0, 1.0)
    return A, b


def check_ops(X, A, b, dtype=torch.float64, tol=1e-13):
    rng = np.random.default_rng(7)
    x = rng.uniform(-0.2, 0.2, size=A.shape[1])
    v = rng.standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    Ax = X.matvec(t(x, dtype))
    assert rel_err(Ax.cpu().numpy(), A @ x) < tol
    y = X.hvp(t(w, dtype), t(v, dtype))
    assert rel_err(y.cpu().numpy(), O.hvp_from_weights(A, w, v)) < tol
    g = X.gradient(Ax, t(O.labels01(b), dtype))
    assert rel_err(g.cpu().numpy(), O.gradient(A, O.labels01(b), x)) < tol
    return x, v, w, Ax, y


# (n, d, mean row length): pass 1 slices over d, pass 2 over n
SHAPES = {
    "accum-both": (3000, 40_000, 6),           # S = 3 / 1: accumulate in both passes
    "slices-x": (2500, 120_000, 5),            # pass 1: 8 slices -> partials + combine
    "tall-t": (40_000, 3000, 3),               # pass 2 over 40 K rows of X^T, pass 1 many rows
    "long-tiles": (1200, 20_000, 30),          # mean per slice 15 -> 16-row tiles
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_window_matches_oracle(shape):
    n, d, mean = SHAPES[shape]
    A, b = skewed(n, d, mean, seed=len(shape))
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    fmt = X.plan_format()
    S1 = -(-d // W64)
    assert fmt["pass1"] == ("window-accum" if S1 <= 4 else "window-slices")
    assert fmt["pass2"] == ("window-accum" if -(-n // W64) <= 4 else "window-slices")
    check_ops(X, A, b)


def test_window_accumulate_is_scipy_bitwise():
    A, b = skewed(3000, 40_000, 6, seed=11)
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format() == {"pass1": "window-accum", "pass2": "window-accum"}
    x, v, w, Ax, y = check_ops(X, A, b)
    np.testing.assert_array_equal(Ax.cpu().numpy(), A @ x)
    np.testing.assert_array_equal(y.cpu().numpy(), O.hvp_from_weights(A, w, v))


def test_window_fp32():
    A, b = skewed(4000, 70_000, 8, seed=5)
    X = krcn.DeviceCSR(A, dtype=torch.float32, fmt=krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format()["pass1"] == "window-accum"      # fp32 window 31,744: S = 3
    check_ops(X, A, b, dtype=torch.float32, tol=1e-5)


def test_window_lanczos():
    """The skewed matrix's few long rows give H outlying eigenvalues, so
    Lanczos loses orthogonality within 12 steps and a 1e-16 HVP perturbation
    moves the oracle's later alphas by ~1e-4 (measured): compare the leading
    alphas / betas with the oracle and the three-term relation
    H v_j = b_{j-1} v_{j-1} + a_j v_j + b_j v_{j+1} for every step."""
    A, b = skewed(2500, 120_000, 5, seed=3)
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    x = np.random.default_rng(1).uniform(-0.2, 0.2, size=A.shape[1])
    w = O.hessian_weights(A, x)
    Ax = X.matvec(t(x))
    g = X.gradient(Ax, t(O.labels01(b)))
    m = 12
    V, al, be, info = X.lanczos(t(w), g, m)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.cpu().numpy(), m)
    assert info.m_eff == m
    assert rel_err(al[:5], al_r[:5]) < 1e-9
    assert rel_err(be[:5], be_r[:5]) < 1e-9
    Vh = V.cpu().numpy()[:m]
    H = lambda q: O.hvp_from_weights(A, w, q)
    scale = np.abs(al).max()
    for j in range(m - 1):
        r = H(Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1] - (be[j - 1] * Vh[j - 1] if j else 0.0)
        assert np.abs(r).max() < 1e-12 * scale, j


def test_window_repeatable():
    A, b = skewed(2500, 120_000, 5, seed=9)
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    v = t(np.random.default_rng(2).standard_normal(A.shape[1]))
    w = t(O.hessian_weights(A, np.zeros(A.shape[1])))
    y0 = X.hvp(w, v).cpu().numpy()
    for _ in range(3):
        np.testing.assert_array_equal(X.hvp(w, v).cpu().numpy(), y0)


@pytest.fixture(scope="module")
def news20():
    from krcn import synth
    return synth.make_problem("news20")


@pytest.mark.parametrize("fmt", [krcn.KRCN_FORMAT_AUTO, krcn.KRCN_FORMAT_WINDOW])
def test_auto_picks_window_on_news20(news20, fmt):
    """Auto: LDS-window slices for X z, the jagged single window for X^T u
    (test_gpu_jag.py); forced window format: the accumulate-mode window for
    X^T u (two windows of u)."""
    A, b = news20
    X = krcn.DeviceCSR(A, fmt=fmt)
    assert X.plan_format() == {"pass1": "window-slices",
                               "pass2": "jagged" if fmt == krcn.KRCN_FORMAT_AUTO else "window-accum"}
    x = np.full(A.shape[1], 0.5)
    v = np.random.default_rng(3).standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    y = X.hvp(t(w), t(v)).cpu().numpy()
    assert rel_err(y, O.hvp_from_weights(A, w, v)) < 1e-13


@pytest.mark.parametrize("mode", ["rows", "cols"])
def test_window_shard_modes_single_rank(mode):
    """The sharded code paths (raw partial passes + all-reduce + elementwise
    epilogues; the Lanczos without the fused step B) over window plans, on a
    1-rank RCCL communicator: must reproduce the unsharded results."""
    from krcn import _lib
    from krcn.dist import Communicator
    A, b = skewed(2500, 120_000, 5, seed=21)
    code = {"rows": _lib.KRCN_SHARD_ROWS, "cols": _lib.KRCN_SHARD_COLS}[mode]
    comm = Communicator(1, 0, torch.device(DEV, 0), Communicator.unique_id())
    try:
        X = krcn.DeviceCSR(A, shard_mode=code, fmt=krcn.KRCN_FORMAT_WINDOW)
        X.attach_comm(comm)
        assert X.plan_format()["pass1"] == "window-slices"
        x, v, w, Ax, y = check_ops(X, A, b)
        X0 = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
        g = X0.gradient(X0.matvec(t(x)), t(O.labels01(b)))
        _, al0, be0, _ = X0.lanczos(t(w), g, 6)
        _, al, be, info = X.lanczos(t(w), g, 6)
        assert info.m_eff == 6
        assert rel_err(al, al0) < 1e-10 and rel_err(be, be0) < 1e-10
    finally:
        comm.close()


def test_lanczos_bitwise_repeated_fused_calls():
    """Repeated fused calls on one handle (window-slice pass 1 with step B,
    pass 2 re-forming z_j) reuse the same workspace: alphas, betas and the
    basis are bitwise the same in every call (no state leaks between calls;
    round 2's w placement probe, which varied the w buffer over calls 1..4,
    was removed in round 3)."""
    A, b = skewed(2500, 120_000, 5, seed=13)
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format()["pass1"] == "window-slices"      # the fused step B runs
    x = np.random.default_rng(4).uniform(-0.2, 0.2, size=A.shape[1])
    w = t(O.hessian_weights(A, x))
    g = X.gradient(X.matvec(t(x)), t(O.labels01(b)))
    ref = None
    for call in range(7):
        V, al, be, info = X.lanczos(w, g, 16)
        out = (V.cpu().numpy(), np.asarray(al), np.asarray(be))
        if ref is None:
            ref = out
            continue
        for a_, r_ in zip(out, ref):
            np.testing.assert_array_equal(a_, r_, err_msg=f"call {call}")


def test_accumulate_plan_grid_beyond_2048_partials():
    """A tall, narrow X^T (d = 14 M columns of X, n = 1,000 rows) makes the
    accumulate-mode pass-2 plan add blocks until each holds <= 96 tiles: over
    2,048 of them.  The Lanczos step A reduces one partial per block, so the
    partials buffers must be sized to the plan's grid (they
    used to hold 2,048 entries and the alphas came from memory past the end)."""
    from krcn import synth
    A, b = synth.make_problem(None, seed=17, n=1000, d=14_000_000, nnz=14_000_000)
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format()["pass2"] == "window-accum"
    assert X.plan_info()["pass2"][3] > 2048
    x = np.full(A.shape[1], 0.5)
    w = O.hessian_weights(A, x)
    g = X.gradient(X.matvec(t(x)), t(O.labels01(b)))
    m = 5
    _, al, be, info = X.lanczos(t(w), g, m)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.cpu().numpy(), m)
    assert info.m_eff == m
    assert rel_err(al, al_r) < 1e-10 and rel_err(be, be_r) < 1e-10


def _xt_problem(n, d, nnz, seed, skew=False):
    from krcn import synth
    return synth.make_problem(None, seed=seed, n=n, d=d, nnz=nnz, skew=skew)


@pytest.mark.parametrize("case", ["w8a-like", "skewed", "breakdown"])
def test_one_piece_fused_xt_lanczos(case):
    """One-piece window-accum plans (d <= 1024: w8a's d = 300) keep a
    column-major copy of each block's rows (PassPlan::xt): the fused Lanczos
    pass 1 forms every block's share of X^T u from the u of its rows in LDS
    (EpiLz1X: chunks of 4 elements of a column in row order, then the
    column's chunks in order), and pass 2 is only k_xt_combine over the block
    partials with step A.  That is not csc_matvec's order: alphas / betas at
    rel 1e-11 against the oracle, the three-term relation at 1e-12, and
    bitwise repeatable.  `breakdown`: 5 live columns of 40 (the rest empty),
    so the Krylov space closes after 5 steps and the reference's absolute
    |beta| < 1e-6 truncation runs."""
    import scipy.sparse as sp_
    n, d, nnz, skew, m = {"w8a-like": (50_000, 300, 580_000, False, 10),
                          "skewed": (30_000, 700, 600_000, True, 12),
                          "breakdown": (20_000, 5, 60_000, False, 12)}[case]
    A, b = _xt_problem(n, d, nnz, seed=31 + d, skew=skew)
    if case == "breakdown":
        A = sp_.hstack([A, sp_.csr_matrix((n, 35))]).tocsr()
        A.sort_indices()
        d = A.shape[1]
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_AUTO if case == "w8a-like" else krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format()["pass1"] == "window-accum"
    x = np.random.default_rng(5).uniform(-0.2, 0.2, size=d)
    w = O.hessian_weights(A, x)
    g = X.gradient(X.matvec(t(x)), t(O.labels01(b)))
    V, al, be, info = X.lanczos(t(w), g, m)
    V_r, al_r, be_r, ret = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.cpu().numpy(), m)
    k = info.m_eff
    assert k == len(al_r) and rel_err(al, al_r) < 1e-11
    if k > 1:
        assert rel_err(be, be_r) < 1e-11
    if case == "breakdown":
        assert info.breakdown and k < m
    else:
        assert k == m
        Vh = V.cpu().numpy()[:m]
        H = lambda q: O.hvp_from_weights(A, w, q)
        scale = np.abs(al).max()
        for j in range(m - 1):
            r = H(Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1] - (be[j - 1] * Vh[j - 1] if j else 0.0)
            assert np.abs(r).max() < 1e-12 * scale, j
    V2, al2, be2, _ = X.lanczos(t(w), g, m)
    np.testing.assert_array_equal(np.asarray(al2), np.asarray(al))
    np.testing.assert_array_equal(V2.cpu().numpy()[:k], V.cpu().numpy()[:k])   # (rows past m_eff: unused)


def test_one_piece_fused_xt_lanczos_fp32():
    A, b = _xt_problem(50_000, 300, 580_000, seed=77)
    X = krcn.DeviceCSR(A, dtype=torch.float32)
    assert X.plan_format()["pass1"] == "window-accum"
    x = np.random.default_rng(6).uniform(-0.2, 0.2, size=A.shape[1])
    w = O.hessian_weights(A, x)
    g = X.gradient(X.matvec(t(x, torch.float32)), t(O.labels01(b), torch.float32))
    _, al, be, info = X.lanczos(t(w, torch.float32), g, 8)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.double().cpu().numpy(), 8)
    assert info.m_eff == 8
    assert rel_err(al[:4], al_r[:4]) < 1e-4 and rel_err(be[:4], be_r[:4]) < 1e-4


@pytest.mark.parametrize("case", ["85x3", "8x32"])
def test_slices_with_empty_row_chunks(case):
    """Window slices whose blocks split a slice's tiles kpb ways (85 slices x 3
    blocks, 8 x 32) on matrices with fewer tiles than kpb: every slice,
    slice 0 included, has blocks with an empty row chunk (WinSeg{slice, 0, 0,
    0}), which load no tiles but still store their share of z_j in the fused
    Lanczos prologue (the tile-base load of such a block
    used to index tb[-1]).  Ops at 1e-13, Lanczos alphas / betas against the
    oracle at 1e-11 and the three-term relation of the stored basis."""
    n, d, mean = {"85x3": (20, 1_300_000, 2000), "8x32": (300, 100_000, 40)}[case]
    A, b = skewed(n, d, mean, seed=21, long_rows=())
    X = krcn.DeviceCSR(A, fmt=krcn.KRCN_FORMAT_WINDOW)
    assert X.plan_format()["pass1"] == "window-slices"
    S, _, tiles, grid = X.plan_info()["pass1"]
    assert S * (3 if case == "85x3" else 32) == grid and tiles < grid // S
    x, v, w, Ax, y = check_ops(X, A, b)
    g = X.gradient(Ax, t(O.labels01(b)))
    m = 8
    V, al, be, info = X.lanczos(t(w), g, m)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g.cpu().numpy(), m)
    assert info.m_eff == m
    assert rel_err(al, al_r) < 1e-11 and rel_err(be, be_r) < 1e-11
    Vh = V.cpu().numpy()[:m]
    scale = np.abs(al).max()
    for j in range(m - 1):
        r = (O.hvp_from_weights(A, w, Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1]
             - (be[j - 1] * Vh[j - 1] if j else 0.0))
        assert np.abs(r).max() < 1e-12 * scale, j
