"""Jagged lane-per-row format (krcn_jag.hpp): one lane owns a row, elements
stored level by level, the gathered vector in LDS as one window (S = 1) or as
two double-buffered windows walked by every block (S > 1).

Bitwise claims: every row is summed left to right over its column-sorted
CSR row, slices in order, multiply and add separate — scipy's csr_matvec /
csc_matvec order — so Ax, X^T u and the HVP equal the oracle's scipy results
bit for bit, whatever the slicing.  Exceptions, at 1e-13: plans with slice
groups (per-group partials), and single-window rows longer than kJagLong = 32
elements, which leave the lane-per-row units and are summed by whole waves
(128-element tasks, a butterfly per task, the tasks in order).  Reference: the oracle (scipy), fp64; fp32
against the fp64 reference at the fp32 bound of DESIGN §4.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import krcn
import krcn_oracle as O
from conftest import rel_err
from test_gpu_tiling import long_row_matrix

pytestmark = pytest.mark.gpu
DEV = "cuda"
JAG = krcn.KRCN_FORMAT_JAG


def t(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def check_bitwise(A, seed=0, exact=True):
    """exact=False: a plan with slice groups (per-group partials) — 1e-13."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.3, 0.3, size=A.shape[1])
    v = rng.standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    X = krcn.DeviceCSR(A, fmt=JAG)
    assert X.plan_format() == {"pass1": "jagged", "pass2": "jagged"}
    u = rng.standard_normal(A.shape[0])
    pairs = [(X.matvec(t(x)), A @ x), (X.rmatvec(t(u)), (A.T @ u) / A.shape[0]),
             (X.hvp(t(w), t(v)), O.hvp_from_weights(A, w, v)),
             (X.hvp(t(w), t(v), l2=0.01), O.hvp_from_weights(A, w, v, l2=0.01))]
    for got, ref in pairs:
        if exact:
            np.testing.assert_array_equal(got.cpu().numpy(), ref)
        else:
            assert rel_err(got.cpu().numpy(), ref) < 1e-13
    return X


def capped_rows(A, cap):
    """A with every row cut to its first `cap` nonzeros."""
    A = A.tocsr(copy=True)
    lens = np.minimum(np.diff(A.indptr), cap)
    keep = np.concatenate([np.arange(A.indptr[r], A.indptr[r] + lens[r]) for r in range(A.shape[0])])
    ptr = np.concatenate([[0], np.cumsum(lens)])
    return sp.csr_matrix((A.data[keep], A.indices[keep], ptr), shape=A.shape)


def test_single_window_short_rows_bitwise():
    """Both passes fit one window (9,000 / 3,000 entries); rows AND columns
    of 0..32 nonzeros (levels 17..32 run the overflow loop; nothing goes to
    the long-row path), empty rows and columns: bit for bit scipy."""
    A, _ = long_row_matrix()
    A = capped_rows(capped_rows(A, 32).T.tocsr(), 32).T.tocsr()
    A.sort_indices()
    X = check_bitwise(A)
    info = X.plan_info()
    assert info["pass1"][0] == 1 and info["pass2"][0] == 1


def test_single_window_long_rows():
    """Rows of 0..5,000 nonzeros in one window (X rows of 509..5,000; X^T rows
    of the 40 hot columns in the hundreds): rows over 32 elements are summed
    apart by whole waves (jag_long_rows: 1..40 tasks a row), the rest in the
    lane-per-row units — value, X^T u, HVP at 1e-13 and the Lanczos
    recurrence at 1e-11 against the oracle over m = 12 (on this matrix a
    1e-16 relative perturbation of the HVP moves the oracle's alphas by
    3.5e-15 at m = 12 and by 0.26 at m = 20: the recurrence itself is
    unstable past m ~ 14)."""
    A, _ = long_row_matrix()
    for cap in (255, None):
        Ac = capped_rows(A, cap) if cap else A
        X = check_bitwise(Ac, exact=False)
        info = X.plan_info()
        assert info["pass1"][0] == 1 and info["pass2"][0] == 1
    rng = np.random.default_rng(12)
    w = O.hessian_weights(A, rng.uniform(-0.3, 0.3, size=A.shape[1]))
    g = rng.standard_normal(A.shape[1])
    _, al, be, _ = X.lanczos(t(w), t(g), 12)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g, 12)
    assert rel_err(al, al_r) < 1e-11 and rel_err(be, be_r) < 1e-11


def test_skewed_news20_shape_auto():
    """news20-shaped, skewed (lognormal rows, power-law columns: X^T rows up to
    16,563 nonzeros, 25 K of them over 32): the automatic choice keeps the
    single-window jagged pass 2 with its long rows summed apart (before, the
    plan was refused and pass 2 fell back to a lane-per-row window pass that
    took 670 us a launch); X^T u at 1e-13."""
    from krcn import synth
    A, _ = synth.make_problem("news20", skew=True)
    X = krcn.DeviceCSR(A)
    assert X.plan_format()["pass2"] == "jagged"
    u = np.random.default_rng(13).standard_normal(A.shape[0])
    assert rel_err(X.rmatvec(t(u)).cpu().numpy(), (A.T @ u) / A.shape[0]) < 1e-13


def test_skewed_rcv1_shape_auto():
    """rcv1-shaped, skewed (power-law columns: X^T rows up to thousands of
    nonzeros).  u (20,242 fp64 entries) leaves 206 task partials of LDS past
    the window, fewer than the 256 a block used to reserve, so round 5 refused
    the jagged plan and pass 2 ran sorted tiles at 318 us a launch
    (profiles/r06s_bench_rcv1_skew.json); the rows over 254 elements now go to
    long-row tasks, as many a block as fit.  X^T u at 1e-13 (long rows are
    summed by wave trees), and the Lanczos recurrence (m = 10) against the
    oracle at 1e-11.  Pass 1 (sorted tiles) takes its lanes from the
    nonzero-weighted mean row (weighted 189 against a mean of 71, 8 slices:
    L = 8; profiles/r06aa_rcv1skew_lanes.txt), while the uniform rcv1 keeps
    the plain slice mean's L = 1."""
    from krcn import synth
    A, b = synth.make_problem("rcv1", skew=True)
    X = krcn.DeviceCSR(A)
    assert X.plan_format()["pass2"] == "jagged"
    if X.plan_format()["pass1"] == "sorted":
        assert X.plan_info()["pass1"][1] == 8
        Au, _ = synth.make_problem("rcv1")
        Xu = krcn.DeviceCSR(Au)
        if Xu.plan_format()["pass1"] == "sorted":
            assert Xu.plan_info()["pass1"][1] == 1
    u = np.random.default_rng(15).standard_normal(A.shape[0])
    assert rel_err(X.rmatvec(t(u)).cpu().numpy(), (A.T @ u) / A.shape[0]) < 1e-13
    x = np.full(A.shape[1], 0.5)
    Ax = X.matvec(t(x))
    w = X.weights(Ax)
    g = X.gradient(Ax, t(O.labels01(b)))
    _, al, be, info = X.lanczos(w, g, 10)
    wh = O.hessian_weights(A, x)
    _, al_r, be_r, _ = O.lanczos(lambda v: O.hvp_from_weights(A, wh, v), g.cpu().numpy(), 10)
    assert info.m_eff == 10
    assert rel_err(al, al_r) < 1e-11 and rel_err(be, be_r) < 1e-11


def test_long_rows_in_a_nearly_full_window():
    """A window of 20,400 fp64 entries leaves 48 task partials of LDS: a row of
    300 elements (three tasks) is summed apart and the plan holds."""
    rng = np.random.default_rng(14)
    n, d = 500, 20_400
    rows = [np.full(6, i) for i in range(n)] + [np.full(300, 7)]
    cols = [rng.choice(d, size=6, replace=False) for _ in range(n)] + [rng.choice(d, size=300, replace=False)]
    A = sp.csr_matrix((rng.uniform(-1, 1, size=sum(map(len, cols))), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n, d))
    A.sum_duplicates()
    A.sort_indices()
    X = krcn.DeviceCSR(A, fmt=JAG)
    assert X.plan_format()["pass1"] == "jagged"
    x = rng.uniform(-0.3, 0.3, size=d)
    assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13


def test_too_long_rows_rejected():
    """Long rows need LDS past the window for their task partials: with the
    window all but full (20,440 of 20,448 fp64 entries: 8 partial slots, fewer
    than one a wave) a row of more than 255 elements cannot be held by the
    8-bit lane counts, so forcing the format fails loudly and the automatic
    choice falls back (results still correct)."""
    rng = np.random.default_rng(14)
    n, d = 500, 20_440
    rows = [np.full(6, i) for i in range(n)] + [np.full(300, 7)]
    cols = [rng.choice(d, size=6, replace=False) for _ in range(n)] + [rng.choice(d, size=300, replace=False)]
    A = sp.csr_matrix((rng.uniform(-1, 1, size=sum(map(len, cols))), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n, d))
    A.sum_duplicates()
    A.sort_indices()
    with pytest.raises(krcn.KrcnError):
        krcn.DeviceCSR(A, fmt=JAG).plan_info()
    x = rng.uniform(-0.3, 0.3, size=d)
    X = krcn.DeviceCSR(A)
    assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13


def test_accumulate_many_slices():
    """d = 100,000 columns: pass 1 walks 11 double-buffered slices of 9,200
    entries; pass 2 (X^T, 2,500 columns) one window.  With 40 row groups the
    plan splits the slices into groups (test_slice_groups): not scipy's
    order, 1e-13."""
    from krcn import synth
    A, _ = synth.make_problem(None, n=2500, d=100_000, nnz=30_000)
    X = check_bitwise(A, seed=1, exact=False)
    assert X.plan_info()["pass1"][0] == 11


def test_accumulate_both_passes_and_tail_slice():
    """Both passes sliced; column counts that leave a short last slice and an
    odd vector length (the window's last 16-byte piece crosses the end)."""
    from krcn import synth
    A, _ = synth.make_problem(None, n=45_001, d=61_237, nnz=270_000)
    X = check_bitwise(A, seed=2)
    info = X.plan_info()
    assert info["pass1"][0] > 1 and info["pass2"][0] > 1


def test_slice_groups():
    """Few rows next to a wide gathered vector (a rank of a row-sharded synth
    run has 1/N of the rows but the whole d-vector): the accumulate plan
    splits the slices into 8 groups (block b: group b % 8, a group per XCD),
    each block walks 1/8 of the windows, and the per-group partial row sums
    are combined in group order — so the row sums are no longer scipy's
    order: 1e-13 against the oracle, and the Lanczos recurrence at 1e-11."""
    from krcn import synth
    A, b = synth.make_problem(None, n=70_000, d=400_000, nnz=2_800_000)
    X = krcn.DeviceCSR(A, fmt=JAG)
    assert X.plan_format()["pass1"] == "jagged"
    rng = np.random.default_rng(11)
    x = rng.uniform(-0.3, 0.3, size=A.shape[1])
    v = rng.standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13
    assert rel_err(X.hvp(t(w), t(v)).cpu().numpy(), O.hvp_from_weights(A, w, v)) < 1e-13
    g = rng.standard_normal(A.shape[1])
    _, al, be, _ = X.lanczos(t(w), t(g), 20)
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g, 20)
    assert rel_err(al, al_r) < 1e-11 and rel_err(be, be_r) < 1e-11


def test_dense_slices_rejected():
    """Accumulate mode holds <= 128 elements of a 64-row group per slice (the
    products slab): a denser matrix is refused when forced and never chosen
    automatically (results still correct through another format)."""
    from krcn import synth
    A, _ = synth.make_problem(None, n=3000, d=60_000, nnz=600_000)
    with pytest.raises(krcn.KrcnError):
        krcn.DeviceCSR(A, fmt=JAG).plan_info()
    x = np.random.default_rng(4).uniform(-0.3, 0.3, size=A.shape[1])
    X = krcn.DeviceCSR(A)
    assert "jagged" not in X.plan_format()["pass1"]
    assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13


def test_unsorted_rows_fall_back():
    """A CSR whose rows are not column-sorted cannot use the level order
    (it would not be the CSR order): forcing the format fails loudly, the
    automatic choice falls back to another format with correct results."""
    A, _ = long_row_matrix()
    A = capped_rows(A, 255)
    # a short row (long rows are summed apart, in any column order)
    r = int(np.flatnonzero((np.diff(A.indptr) >= 3) & (np.diff(A.indptr) <= 32))[0])
    r0, r1 = A.indptr[r], A.indptr[r + 1]
    A.indices[r0:r1] = A.indices[r0:r1][::-1].copy()
    A.data[r0:r1] = A.data[r0:r1][::-1].copy()
    with pytest.raises(krcn.KrcnError):
        krcn.DeviceCSR(A, fmt=JAG).plan_info()
    x = np.random.default_rng(5).uniform(-0.3, 0.3, size=A.shape[1])
    X = krcn.DeviceCSR(A)
    assert rel_err(X.matvec(t(x)).cpu().numpy(), A @ x) < 1e-13


def test_fp32():
    from krcn import synth
    A, _ = synth.make_problem(None, n=20_000, d=70_000, nnz=80_000)
    rng = np.random.default_rng(6)
    x = rng.uniform(-0.3, 0.3, size=A.shape[1])
    v = rng.standard_normal(A.shape[1])
    w = O.hessian_weights(A, x)
    X = krcn.DeviceCSR(A, dtype=torch.float32, fmt=JAG)
    assert X.plan_format() == {"pass1": "jagged", "pass2": "jagged"}
    y = X.hvp(t(w, torch.float32), t(v, torch.float32)).cpu().numpy()
    assert rel_err(y, O.hvp_from_weights(A, w, v)) < 1e-5
    assert rel_err(X.matvec(t(x, torch.float32)).cpu().numpy(), A @ x) < 1e-5


def test_lanczos_jag_matches_sequential():
    """The Lanczos recurrence over jagged passes against the one over the
    sequential-lane plans: the HVPs agree bit for bit (both scipy's order);
    the v.w / ||z|| reductions are summed per block of each plan's own grid,
    so alphas / betas agree to rounding (measured ~4.5e-16)."""
    from krcn import synth
    A, b = synth.make_problem(None, n=30_000, d=50_000, nnz=180_000)
    x = np.random.default_rng(7).uniform(-0.2, 0.2, size=A.shape[1])
    w = O.hessian_weights(A, x)
    g = np.random.default_rng(8).standard_normal(A.shape[1])
    Xj = krcn.DeviceCSR(A, fmt=JAG)
    Xs = krcn.DeviceCSR(A, lanes=(1, 1), fmt=krcn.KRCN_FORMAT_WAVE)
    Vj, aj, bj, ij = Xj.lanczos(t(w), t(g), 20)
    Vs, as_, bs, is_ = Xs.lanczos(t(w), t(g), 20)
    assert rel_err(aj, as_) < 1e-13 and rel_err(bj, bs) < 1e-13
    _, al_r, be_r, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q), g, 20)
    assert rel_err(aj, al_r) < 1e-11 and rel_err(bj, be_r) < 1e-11


def test_auto_policy_picks_jag_for_news20_pass2():
    """news20 shape: X^T (1.36 M rows of ~6.7) gathers from u (19,996
    entries): one jagged window; pass 1 keeps the LDS-window slices (the fused
    Lanczos step B needs them)."""
    from krcn import synth
    A, _ = synth.make_problem("news20")
    X = krcn.DeviceCSR(A)
    assert X.plan_format() == {"pass1": "window-slices", "pass2": "jagged"}
    rng = np.random.default_rng(9)
    u = rng.standard_normal(A.shape[0])
    np.testing.assert_array_equal(X.rmatvec(t(u)).cpu().numpy(), (A.T @ u) / A.shape[0])


def test_auto_policy_rcv1_pass2_jagged_fp64_only():
    """rcv1 shape: X^T has 47 K rows (738 row groups, fewer than one per wave)
    and gathers from u (20 K entries, one window).  Since round 3 the fp64 X^T
    pass takes the single-window jagged format with blocks of >= 6 groups
    (13.2 -> 11.5 us, profiles/r03_rcv1_jag_ab.txt); pass 1 keeps its sliced
    sorted tiles (the fused step B), and fp32 keeps the sorted X^T pass (the
    jagged one measured slower there).  X^T rows over 32 elements (this
    shape: up to 60) are summed by the long-row tasks, so 1e-13; otherwise
    bitwise scipy."""
    from krcn import synth
    A, _ = synth.make_problem("rcv1")
    X = krcn.DeviceCSR(A)
    assert X.plan_format() == {"pass1": "sorted", "pass2": "jagged"}
    assert X.plan_info()["pass2"][3] < 256                     # fewer blocks than CUs
    u = np.random.default_rng(10).standard_normal(A.shape[0])
    y = X.rmatvec(t(u)).cpu().numpy()
    ref = (A.T @ u) / A.shape[0]
    if np.diff(A.tocsc().indptr).max() <= 32:
        np.testing.assert_array_equal(y, ref)
    else:
        assert rel_err(y, ref) < 1e-13
    X32 = krcn.DeviceCSR(A, dtype=torch.float32)
    assert X32.plan_format()["pass2"] != "jagged"
