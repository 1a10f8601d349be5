"""Device Lanczos (cubic.py:77-111) vs the reference's golden outputs.

Tolerances (fp64, three-term, m <= 100): alphas/betas rel 1e-11, basis V
max-abs 1e-9 (SURVEY.md §8c evidence: a 1e-15 HVP perturbation moves them
by <= 1e-15 for m <= 100).  The breakdown quirks must match exactly in
structure: m_eff, which betas are zero, the zero last basis vector, and which
alpha the final Rayleigh quotient overwrites.
"""
import numpy as np
import pytest
import torch

import krcn
import krcn_oracle as O
from conftest import golden_csr, load_golden, rel_err
from krcn import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def device_operator(A, b, x, **plan):
    X = krcn.DeviceCSR(A, **plan)
    Ax = X.matvec(t(x))
    w = X.weights(Ax)
    g = X.gradient(Ax, t(O.labels01(b)))
    return X, w, g


@pytest.mark.parametrize("m", [1, 10])
def test_lanczos_vs_golden(f1, f2, m):
    """f1's operator (n = 257) is ill-conditioned for Lanczos: a 1e-16 relative
    HVP perturbation moves the oracle's V[:, 9] by 8e-9 (alphas/betas by 4e-15),
    so V is compared at 1e-6 and alphas/betas at 1e-11."""
    A = golden_csr(f1)
    X, w, g = device_operator(A, f1["b"], f1["x0"])
    V, al, be, info = X.lanczos(w, g, m)
    assert info.m_eff == m and not info.breakdown and info.hvps == m
    assert rel_err(al, f2[f"alphas_m{m}"]) < 1e-11
    assert rel_err(be, f2[f"betas_m{m}"]) < 1e-11
    Vh = V.cpu().numpy()[:info.m_eff].T
    assert np.abs(Vh - f2[f"V_m{m}"]).max() < 1e-6
    assert abs(info.beta_last - float(f2[f"beta_m{m}"])) <= 1e-11 * max(1e-300, abs(float(f2[f"beta_m{m}"])))
    assert abs(info.gnorm - np.linalg.norm(f2["g"])) <= 1e-13 * np.linalg.norm(f2["g"])


def test_lanczos_three_term_relation(f1):
    """m = 50 on f1 is past the point where rounding decides alphas/betas (a
    1e-16 HVP perturbation changes them by 40 %), so check what the
    recurrence guarantees instead: H v_j = b_{j-1} v_{j-1} + a_j v_j + b_j v_{j+1}
    with the device's own basis, unit vectors, local orthogonality."""
    A = golden_csr(f1)
    x = f1["x0"]
    X, w, g = device_operator(A, f1["b"], x)
    V, al, be, info = X.lanczos(w, g, 50)
    Vh = V.cpu().numpy()[:info.m_eff]
    wh = O.hessian_weights(A, x)
    H = lambda v: O.hvp_from_weights(A, wh, v)  # noqa: E731
    hn = max(np.abs(al).max(), np.abs(be).max())
    for j in range(info.m_eff - 1):
        r = H(Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1] - (be[j - 1] * Vh[j - 1] if j else 0)
        assert np.linalg.norm(r) < 1e-12 * hn
        assert abs(np.linalg.norm(Vh[j]) - 1) < 1e-14
        assert abs(Vh[j] @ Vh[j + 1]) < 1e-12
    assert abs(al[-1] - Vh[-1] @ H(Vh[-1])) < 1e-12 * hn


@pytest.mark.parametrize("r,ms", [(1, (2, 3, 5)), (3, (4, 5, 10))])
def test_lanczos_breakdown_quirks(f2, r, ms):
    A = golden_csr(f2, f"r{r}_")
    X, w, g = device_operator(A, f2[f"r{r}_b"], np.full(A.shape[1], 0.5))
    for m in ms:
        key = f"r{r}_m{m}"
        V, al, be, info = X.lanczos(w, g, m)
        Vref = f2[f"{key}_V"]
        assert info.breakdown == 1 and info.j_break == r - 1
        assert info.m_eff == Vref.shape[1]
        assert al.shape == f2[f"{key}_alphas"].shape and be.shape == f2[f"{key}_betas"].shape
        assert rel_err(al, f2[f"{key}_alphas"]) < 1e-11
        np.testing.assert_allclose(be, f2[f"{key}_betas"], rtol=1e-11, atol=0)
        Vh = V.cpu().numpy()[:info.m_eff].T
        assert np.abs(Vh - Vref).max() < 1e-12
        if m == r + 1:                       # breakdown at j == m-2: zero last column kept
            assert np.all(Vh[:, -1] == 0) and be[-1] == 0
        assert info.beta_last < 1e-6


# Plans whose pass 1 runs step B of each Lanczos step itself:
#  sorted: sorted tiles over 8 column slices (the gathers form z = w - alpha v,
#          the blocks store their share of z and its norm partials; the slice
#          combine settles beta);
#  small:  the one-piece LDS window (d <= 1024, window-accum): every block
#          forms all of z and beta itself, no step-B launch, no combine.
#  two_launch: unsliced sorted pass 1 (z_j formed in the gathers, u' = w X z_j
#          stored) + single-window jagged pass 2 whose blocks settle beta and
#          scale their window (SrcLzU): two launches a step, no combine.
FUSED_PLANS = {"sorted": dict(slicing=8, fmt=krcn.KRCN_FORMAT_SORTED),
               "small": dict(fmt=krcn.KRCN_FORMAT_WINDOW),
               "two_launch": dict(pass_formats=(krcn.KRCN_FORMAT_SORTED, krcn.KRCN_FORMAT_JAG))}


def check_fused_plan(X, kind):
    info, fmt = X.plan_info(), X.plan_format()
    if kind == "sorted":
        assert info["pass1"][0] == -8
    elif kind == "two_launch":
        assert info["pass1"][0] == -1 and fmt["pass2"] == "jagged" and info["pass2"][0] == 1
    else:
        assert fmt["pass1"] == "window-accum" and info["pass1"][0] == 1 and X.d <= 1024


@pytest.mark.parametrize("kind", sorted(FUSED_PLANS))
@pytest.mark.parametrize("m", [1, 10])
def test_lanczos_fused_step_b_vs_golden(f1, f2, m, kind):
    A = golden_csr(f1)
    X, w, g = device_operator(A, f1["b"], f1["x0"], **FUSED_PLANS[kind])
    check_fused_plan(X, kind)
    V, al, be, info = X.lanczos(w, g, m)
    assert info.m_eff == m and not info.breakdown and info.hvps == m
    assert rel_err(al, f2[f"alphas_m{m}"]) < 1e-11
    assert rel_err(be, f2[f"betas_m{m}"]) < 1e-11
    Vh = V.cpu().numpy()[:info.m_eff].T
    assert np.abs(Vh - f2[f"V_m{m}"]).max() < 1e-6
    assert abs(info.beta_last - float(f2[f"beta_m{m}"])) <= 1e-11 * max(1e-300, abs(float(f2[f"beta_m{m}"])))
    assert abs(info.gnorm - np.linalg.norm(f2["g"])) <= 1e-13 * np.linalg.norm(f2["g"])


@pytest.mark.parametrize("kind", sorted(FUSED_PLANS))
@pytest.mark.parametrize("r,ms", [(1, (2, 3, 5)), (3, (4, 5, 10))])
def test_lanczos_fused_step_b_breakdown_quirks(f2, r, ms, kind):
    A = golden_csr(f2, f"r{r}_")
    X, w, g = device_operator(A, f2[f"r{r}_b"], np.full(A.shape[1], 0.5), **FUSED_PLANS[kind])
    check_fused_plan(X, kind)
    for m in ms:
        key = f"r{r}_m{m}"
        V, al, be, info = X.lanczos(w, g, m)
        Vref = f2[f"{key}_V"]
        assert info.breakdown == 1 and info.j_break == r - 1
        assert info.m_eff == Vref.shape[1]
        assert rel_err(al, f2[f"{key}_alphas"]) < 1e-11
        np.testing.assert_allclose(be, f2[f"{key}_betas"], rtol=1e-11, atol=0)
        Vh = V.cpu().numpy()[:info.m_eff].T
        assert np.abs(Vh - Vref).max() < 1e-12
        if m == r + 1:
            assert np.all(Vh[:, -1] == 0) and be[-1] == 0
        assert info.beta_last < 1e-6


# Window-slices pass 1 (news20's plan) runs the early-alpha step
# (krcn_kernels.hpp EpiLz2E): the slice combine also forms the partials of
# (X v_j).(w X v_j), pass 2 settles alpha_j from them (and the previous pass
# 2's z_j . v_{j-1}) in its prologue and runs step B in its epilogue.  The
# golden operators are too narrow for a sliced window (d <= 1,024 takes the
# one-piece plan), so their columns are padded with empty ones to
# d = 140,000: the padded operator acts as the original on the first d
# columns and as zero on the rest, so the reference's outputs hold with zero
# rows appended to V.  Pass 2 runs either as the single-window jagged pass
# (news20's) or the accumulate window pass; early_sorted is rcv1's plan
# family (sorted tiles over 8 column slices, jagged pass 2).
EARLY_PLANS = {"early_jag": dict(pass_formats=(krcn.KRCN_FORMAT_WINDOW, krcn.KRCN_FORMAT_JAG)),
               "early_win": dict(fmt=krcn.KRCN_FORMAT_WINDOW),
               "early_sorted": dict(slicing=8, pass_formats=(krcn.KRCN_FORMAT_SORTED, krcn.KRCN_FORMAT_JAG))}
D_PAD = 140_000


def pad_cols(A, d):
    import scipy.sparse as sp
    return sp.csr_matrix((A.data, A.indices, A.indptr), shape=(A.shape[0], d))


def early_operator(A0, b, x0, kind):
    d0 = A0.shape[1]
    X, w, g = device_operator(pad_cols(A0, D_PAD), b, np.concatenate([x0, np.zeros(D_PAD - d0)]),
                              **EARLY_PLANS[kind])
    fmt = X.plan_format()
    if kind == "early_sorted":   # rcv1's plan family: sorted tiles over 8 column slices
        assert X.plan_info()["pass1"][0] == -8 and fmt["pass2"] == "jagged"
    else:
        assert fmt["pass1"] == "window-slices"
        assert fmt["pass2"] == ("jagged" if kind == "early_jag" else "window-accum")
    return X, w, g


def check_padded_basis(V, m_eff, Vref, tol):
    Vh = V.cpu().numpy()[:m_eff].T
    d0 = Vref.shape[0]
    assert np.abs(Vh[:d0] - Vref).max() < tol
    assert np.all(Vh[d0:] == 0)
    return Vh[:d0]


@pytest.mark.parametrize("kind", sorted(EARLY_PLANS))
@pytest.mark.parametrize("m", [1, 10, 50])
def test_lanczos_early_alpha_vs_golden(f1, f2, m, kind):
    """alphas / betas at 1e-11 for m = 1 and 10 (as the other plans); at m = 50,
    past where rounding decides them on f1 (test_lanczos_three_term_relation),
    the three-term relation with the device's basis, unit vectors and local
    orthogonality (what the z.v term of alpha keeps)."""
    A0 = golden_csr(f1)
    X, w, g = early_operator(A0, f1["b"], f1["x0"], kind)
    V, al, be, info = X.lanczos(w, g, m)
    assert info.m_eff == m and not info.breakdown and info.hvps == m
    assert abs(info.gnorm - np.linalg.norm(f2["g"])) <= 1e-13 * np.linalg.norm(f2["g"])
    if m <= 10:
        assert rel_err(al, f2[f"alphas_m{m}"]) < 1e-11
        assert rel_err(be, f2[f"betas_m{m}"]) < 1e-11
        check_padded_basis(V, m, f2[f"V_m{m}"], 1e-6)
        assert abs(info.beta_last - float(f2[f"beta_m{m}"])) <= 1e-11 * max(1e-300, abs(float(f2[f"beta_m{m}"])))
        return
    Vh = V.cpu().numpy()[:m]
    assert np.all(Vh[:, A0.shape[1]:] == 0)
    Vh = Vh[:, :A0.shape[1]]
    wh = O.hessian_weights(A0, f1["x0"])
    H = lambda v: O.hvp_from_weights(A0, wh, v)  # noqa: E731
    hn = max(np.abs(al).max(), np.abs(be).max())
    for j in range(m - 1):
        r = H(Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1] - (be[j - 1] * Vh[j - 1] if j else 0)
        assert np.linalg.norm(r) < 1e-12 * hn
        assert abs(np.linalg.norm(Vh[j]) - 1) < 1e-14
        assert abs(Vh[j] @ Vh[j + 1]) < 1e-12
    assert abs(al[-1] - Vh[-1] @ H(Vh[-1])) < 1e-12 * hn


@pytest.mark.parametrize("kind", sorted(EARLY_PLANS))
@pytest.mark.parametrize("r,ms", [(1, (2, 3, 5)), (3, (4, 5, 10))])
def test_lanczos_early_alpha_breakdown_quirks(f2, r, ms, kind):
    """The breakdown is detected one launch later than on the other plans
    (pass 1 of step j settles beta_{j-1}); alphas[j_break] is still
    overwritten by the Rayleigh quotient, the basis truncated, and a
    breakdown at j = m-2 keeps the zero last column."""
    A0 = golden_csr(f2, f"r{r}_")
    X, w, g = early_operator(A0, f2[f"r{r}_b"], np.full(A0.shape[1], 0.5), kind)
    for m in ms:
        key = f"r{r}_m{m}"
        V, al, be, info = X.lanczos(w, g, m)
        Vref = f2[f"{key}_V"]
        assert info.breakdown == 1 and info.j_break == r - 1
        assert info.m_eff == Vref.shape[1]
        assert al.shape == f2[f"{key}_alphas"].shape and be.shape == f2[f"{key}_betas"].shape
        assert rel_err(al, f2[f"{key}_alphas"]) < 1e-11
        np.testing.assert_allclose(be, f2[f"{key}_betas"], rtol=1e-11, atol=0)
        Vh = check_padded_basis(V, info.m_eff, Vref, 1e-12)
        if m == r + 1:
            assert np.all(Vh[:, -1] == 0) and be[-1] == 0
        assert info.beta_last < 1e-6


L2 = 0.01


@pytest.mark.parametrize("kind", sorted(EARLY_PLANS))
@pytest.mark.parametrize("m", [1, 5, 10])
def test_lanczos_early_alpha_l2(f1, kind, m):
    """l2 != 0 on the early-alpha plans: the step forms
    alpha_j = (X v).(w X v) / n + l2 - z_j . v_{j-1}, i.e. it writes the
    reference's l2 v.v (loss.py:302 inside cubic.py:93-94) as l2 because v_j is
    unit to rounding.  alphas / betas against the oracle's three-term Lanczos
    over hvp_from_weights(.., l2 = 0.01) at 1e-11 (the golden tolerance)."""
    A0 = golden_csr(f1)
    X, w, g = early_operator(A0, f1["b"], f1["x0"], kind)
    V, al, be, info = X.lanczos(w, g, m, l2=L2)
    d0 = A0.shape[1]
    wh = O.hessian_weights(A0, f1["x0"])
    gh = g.cpu().numpy()
    assert np.all(gh[d0:] == 0)
    Vr, al_r, be_r, beta_r = O.lanczos(lambda v: O.hvp_from_weights(A0, wh, v, l2=L2), gh[:d0], m)
    assert info.m_eff == m and not info.breakdown
    assert rel_err(al, al_r) < 1e-11
    assert rel_err(be, be_r) < 1e-11
    check_padded_basis(V, m, Vr, 1e-6)
    assert abs(info.beta_last - float(beta_r)) <= 1e-11 * max(1e-300, abs(float(beta_r)))


def test_lanczos_fused_small_w8a_shape():
    """w8a's shape (d = 300, binary values) through the auto plan, whose pass 1
    is the one-piece window.  The recurrence loses conditioning within m = 10
    on this shape (test_gpu_configs.py header), so the leading six alphas /
    betas against the oracle at 1e-11, and every step through the three-term
    relation with the device's own basis."""
    A, b = synth.make_problem("w8a", n=20_000, nnz=230_000)
    x = np.random.default_rng(5).uniform(-0.2, 0.2, size=A.shape[1])
    X, w, g = device_operator(A, b, x)
    assert X.plan_format()["pass1"] == "window-accum"
    V, al, be, info = X.lanczos(w, g, 10)
    wh = O.hessian_weights(A, x)
    H = lambda q: O.hvp_from_weights(A, wh, q)  # noqa: E731
    _, al_r, be_r, _ = O.lanczos(H, g.cpu().numpy(), 10)
    assert rel_err(al[:6], al_r[:6]) < 1e-11 and rel_err(be[:6], be_r[:6]) < 1e-11
    Vh = V.cpu().numpy()[:info.m_eff]
    scale = np.abs(al).max()
    for j in range(info.m_eff - 1):
        r = H(Vh[j]) - al[j] * Vh[j] - be[j] * Vh[j + 1] - (be[j - 1] * Vh[j - 1] if j else 0.0)
        assert np.abs(r).max() < 1e-12 * scale, j


def test_lanczos_deterministic(f1):
    A = golden_csr(f1)
    X, w, g = device_operator(A, f1["b"], f1["x1"])
    V1, a1, b1, _ = X.lanczos(w, g, 30)
    V1 = V1.clone()
    V2, a2, b2, _ = X.lanczos(w, g, 30)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(b1, b2)
    assert torch.equal(V1, V2)


def test_lanczos_reorth_matches_cgs2_oracle(f1):
    A = golden_csr(f1)
    x = f1["x0"]
    X, w, g = device_operator(A, f1["b"], x)
    wh = O.hessian_weights(A, x)
    gh = g.cpu().numpy()
    _, al_ref, be_ref, _ = O.lanczos_cgs2(lambda v: O.hvp_from_weights(A, wh, v), gh, 40)
    V, al, be, info = X.lanczos(w, g, 40, reorth=True)
    assert info.m_eff == len(al_ref)
    assert rel_err(al, al_ref) < 1e-10
    assert rel_err(be, be_ref) < 1e-10
    Vh = V.cpu().numpy()[:info.m_eff]
    assert np.abs(Vh @ Vh.T - np.eye(info.m_eff)).max() < 1e-12


def test_rcv1_shape_alphas_betas():
    f = load_golden("f5_rcv1.npz")
    A, b = synth.make_problem("rcv1")
    X, w, g = device_operator(A, b, np.full(A.shape[1], 0.5))
    V, al, be, info = X.lanczos(w, g, int(f["m"]))
    assert info.m_eff == int(f["m"])
    assert rel_err(al, f["alphas"]) < 1e-11
    assert rel_err(be, f["betas"]) < 1e-11
    st = int(f["stride"])
    assert np.abs(V[-1].cpu().numpy()[::st] - f["V_last_sample"]).max() < 1e-9


def test_news20_shape_alphas_betas():
    f = load_golden("f5_news20.npz")
    A, b = synth.make_problem("news20")
    X, w, g = device_operator(A, b, np.full(A.shape[1], 0.5))
    V, al, be, info = X.lanczos(w, g, int(f["m"]))
    assert info.m_eff == 100 and info.hvps == 100
    # measured envelope: a 1e-16 HVP perturbation moves the oracle's m=100
    # alphas/betas by 2e-9 (rcv1 m=50: 7e-16)
    assert rel_err(al, f["alphas"]) < 1e-7
    assert rel_err(be, f["betas"]) < 1e-7


@pytest.mark.parametrize("m", [60, 150])
def test_reorth_rcv1_fp64_and_orthogonality(m):
    """CGS2 (build-only) at rcv1 shape: matches the oracle's CGS2 definition
    and keeps the basis orthonormal to 1e-12.  m = 150 runs the 1 KiB-piece
    sweeps with up to three row ranges per column group (the in-launch
    combine of k_cgs_colsweep)."""
    A, b = synth.make_problem("rcv1")
    x = np.full(A.shape[1], 0.5)
    X, w, g = device_operator(A, b, x)
    wh = O.hessian_weights(A, x)
    _, al_r, be_r, _ = O.lanczos_cgs2(lambda v: O.hvp_from_weights(A, wh, v), g.cpu().numpy(), m)
    V, al, be, info = X.lanczos(w, g, m, reorth=True)
    assert info.m_eff == m
    assert rel_err(al, al_r) < 1e-10
    assert rel_err(be, be_r) < 1e-10
    Vh = V.cpu().numpy()
    assert np.abs(Vh @ Vh.T - np.eye(m)).max() < 1e-12


def test_reorth_wide_rows_fp64():
    """CGS2 on rows of 200,000 fp64 entries at m = 260: the
    1 KiB-piece row sweep cuts such a row into 25 chunks (more than the 16
    that the round-4 partials buffer was sized for: its C k chunk partials ran
    past the end), and sweeps over k > 256 rows split into two row ranges
    (the colsweep's in-launch combine, whose buffer is now sized from the
    launcher's range length).  Against the oracle's CGS2 at 1e-10, basis
    orthonormal to 1e-12.  (The oracle takes ~20 s here.)"""
    A, b = synth.make_problem(None, seed=29, n=3000, d=200_000, nnz=300_000)
    x = np.full(A.shape[1], 0.5)
    X, w, g = device_operator(A, b, x)
    m = 260
    X.reserve(m, reorth=True)
    V, al, be, info = X.lanczos(w, g, m, reorth=True)
    assert info.m_eff == m
    wh = O.hessian_weights(A, x)
    _, al_r, be_r, _ = O.lanczos_cgs2(lambda v: O.hvp_from_weights(A, wh, v), g.cpu().numpy(), m)
    assert rel_err(al, al_r) < 1e-10
    assert rel_err(be, be_r) < 1e-10
    Vh = V.cpu().numpy()
    assert np.abs(Vh @ Vh.T - np.eye(m)).max() < 1e-12


@pytest.mark.parametrize("d,dtype", [(24, torch.float64), (25, torch.float64), (24, torch.float32)])
def test_reorth_breakdown_matches_cgs2_oracle(d, dtype):
    """CGS2 past the Krylov dimension: with d = 24 or 25 columns and m = 40
    the recurrence breaks down (|beta| < tol) at j = d and truncates as the
    reference does (cubic.py:98-109).  d = 24 runs the 1 KiB-piece sweeps with
    step B inside the first sweep (k_cgs_rowdots_vb), whose early return on
    the done flag must leave alphas, betas and V as the separate step B does;
    d = 25 (rows not whole 16-byte vectors) runs the batched kernels."""
    A, b = synth.make_problem(None, seed=7, n=200, d=d, nnz=3000)
    x = np.full(d, 0.5)
    X = krcn.DeviceCSR(A, dtype=dtype)
    Ax = X.matvec(torch.full((d,), 0.5, dtype=dtype, device=DEV))
    w = X.weights(Ax)
    g = X.gradient(Ax, torch.from_numpy(O.labels01(b)).to(DEV, dtype))
    wh = O.hessian_weights(A, x)
    gh = O.gradient(A, O.labels01(b), x)
    Vr, al_r, be_r, _ = O.lanczos_cgs2(lambda v: O.hvp_from_weights(A, wh, v), gh, 40)
    V, al, be, info = X.lanczos(w, g, 40, reorth=True)
    assert info.m_eff == len(al_r) < 40
    tol = 1e-9 if dtype == torch.float64 else 1e-3
    assert rel_err(al, al_r) < tol
    assert rel_err(be, be_r) < tol
    Vh = V.cpu().numpy()[:info.m_eff].astype(np.float64)
    assert np.abs(Vh @ Vh.T - np.eye(info.m_eff)).max() < (1e-12 if dtype == torch.float64 else 1e-5)


def test_reorth_fp32_stress_config():
    """rcv1_stress: fp32 data and basis, CGS2; compared with the fp64 oracle
    CGS2 (fp32 rounding, rel 1e-3) and fp32-level orthogonality."""
    A, b = synth.make_problem("rcv1")
    x = np.full(A.shape[1], 0.5)
    X = krcn.DeviceCSR(A, dtype=torch.float32)
    Ax = X.matvec(torch.full((A.shape[1],), 0.5, dtype=torch.float32, device=DEV))
    w = X.weights(Ax)
    g = X.gradient(Ax, torch.from_numpy(O.labels01(b)).to(DEV, torch.float32))
    m = 120
    V, al, be, info = X.lanczos(w, g, m, reorth=True)
    assert info.m_eff == m
    wh = O.hessian_weights(A, x)
    gh = O.gradient(A, O.labels01(b), x)
    _, al_r, be_r, _ = O.lanczos_cgs2(lambda v: O.hvp_from_weights(A, wh, v), gh, m)
    assert rel_err(al[:40], al_r[:40]) < 1e-3
    assert rel_err(be[:40], be_r[:40]) < 1e-3
    Vh = V.cpu().numpy().astype(np.float64)
    assert np.abs(Vh @ Vh.T - np.eye(m)).max() < 1e-5
