"""The sharded path at BASELINE scale on one GPU: 8 virtual ranks.

`krcn.dist.VirtualShards` cuts the matrix with the same partition an 8-GPU
job uses (`krcn.dist.plan`), gives every rank its own handle in the shard mode
(with the rank-level plans the auto policy picks: jagged slice groups for a
synth row block, unsliced tiles for a news20 column block), its own stream and
host thread, and a communicator of one virtual group: each all-reduce inside
the library is a rendezvous of the rank threads and a device sum in rank order
(include/krcn.h, krcn_comm_create_virtual).  Everything but the transport is
the multi-GPU code path, so these are the parity tests of BASELINE config 5
(synth 2 M x 1 M, 200 M nnz, row-sharded x 8) and of the news20 column split
the scaling run takes, against fixtures the REFERENCE produced on the same
matrices (tests/golden/make_golden.py, f5_<cfg>.npz).

Tolerances as for the unsharded configs (tests/test_gpu_configs.py): the rank
sums change only the order of the d- (rows) or n-length (cols) partial sums.
  value / gradient / HVP: rel 1e-13 / 1e-13 / 1e-12; synth alphas / betas
  1e-11; news20 alphas / betas at the measured m = 100 envelope 1e-7
  (tests/test_gpu_lanczos.py::test_news20_shape_alphas_betas); synth one
  Krylov-CRN step f_k / x_k 1e-10.
Reference: optimizer/loss.py:215-232 (value, gradient), :289-302 (HVP),
optimizer/cubic.py:77-111 (Lanczos), :265-309 (the CRN step).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, rel_err
from krcn import dist as kdist
from krcn import synth
from optimizer.cubic import Cubic_Krylov_LS
from optimizer.loss import LogisticRegression

pytestmark = pytest.mark.gpu
WORLD = 8


def rank_statistics(vs, m):
    """value, gradient, ||g||, one HVP at v = g/||g|| and the m-step Lanczos,
    on every virtual rank at x = 0.5 (the reference's x0, cubic_newton.py:61)."""

    def fn(r):
        X, b = vs.X[r], vs.b[r]
        x = torch.full((X.d,), 0.5, dtype=X.dtype, device=X.device)
        Ax = X.matvec(x)
        val = X.loss_mean(Ax, b)
        g = X.gradient(Ax, b)
        gn = X.diff_norm(g)
        w = X.weights(Ax)
        y = X.hvp(w, (g / gn).contiguous())
        _, al, be, info = X.lanczos(w, g, m)
        return {"value": val, "g": g.cpu().numpy(), "gn": gn, "y": y.cpu().numpy(), "al": al, "be": be,
                "m_eff": info.m_eff, "beta": info.beta_last, "fmt": X.plan_format(), "plan": X.plan_info()}

    return vs.run(fn)


def check(f, res, g, y, lanczos_tol):
    st = int(f["stride"])
    for r in res:
        assert abs(r["value"] - f["value"]) <= 1e-13 * abs(f["value"])
        assert abs(r["gn"] - f["g_norm"]) <= 1e-13 * f["g_norm"]
        assert r["m_eff"] == len(f["alphas"])
        assert rel_err(r["al"], f["alphas"]) < lanczos_tol
        assert rel_err(r["be"], f["betas"]) < lanczos_tol
        assert abs(r["beta"] - float(f["beta"])) <= lanczos_tol * abs(float(f["beta"]))
        # the recurrence is replicated: every rank holds the same scalars
        np.testing.assert_array_equal(r["al"], res[0]["al"])
        np.testing.assert_array_equal(r["be"], res[0]["be"])
    assert rel_err(g[::st], f["g_sample"]) < 1e-13
    assert rel_err(y[::st], f["y_sample"]) < 1e-12
    assert abs(np.linalg.norm(y) - f["y_norm"]) <= 1e-12 * f["y_norm"]


def test_news20_cols_x8():
    f = load_golden("f5_news20.npz")
    A, b = synth.make_problem("news20")
    vs = kdist.VirtualShards(A, b, WORLD, partition="cols")
    try:
        assert vs.mode == "cols"
        res = rank_statistics(vs, int(f["m"]))
    finally:
        vs.close()
    # d-vectors are sharded: the global gradient / HVP is the rank blocks in order
    g = np.concatenate([r["g"] for r in res])
    y = np.concatenate([r["y"] for r in res])
    assert g.shape[0] == A.shape[1]
    check(f, res, g, y, 1e-7)


@pytest.fixture(scope="module")
def synth_problem():
    return synth.make_problem("synth")


def test_synth_rows_x8(synth_problem):
    f = load_golden("f5_synth.npz")
    A, b = synth_problem
    vs = kdist.VirtualShards(A, b, WORLD, partition="rows")
    try:
        assert vs.mode == "rows"
        res = rank_statistics(vs, int(f["m"]))
    finally:
        vs.close()
    # d-vectors are replicated (all-reduced): every rank holds the whole, same bits
    for r in res[1:]:
        np.testing.assert_array_equal(r["g"], res[0]["g"])
        np.testing.assert_array_equal(r["y"], res[0]["y"])
    # a rank's X block gathers the whole d-vector: the auto policy runs its
    # pass 1 in jagged slice groups
    assert res[0]["fmt"]["pass1"] == "jagged"
    check(f, res, res[0]["g"], res[0]["y"], 1e-11)


def test_synth_rows_x8_crn_step(synth_problem):
    """One Krylov-CRN step (cubic.py:265-309) on 8 virtual ranks: the line
    search, x + V s and the loss values run through the sharded handles."""
    f = load_golden("f5_synth.npz")
    A, b = synth_problem
    mode, bounds = kdist.plan(A, WORLD, "rows")
    comms = kdist.Communicator.virtual(WORLD, torch.device("cuda", torch.cuda.current_device()))
    specs = [kdist.ShardSpec(A, mode, bounds, r, WORLD, comms[r]) for r in range(WORLD)]
    dev = torch.device("cuda", torch.cuda.current_device())
    streams = [torch.cuda.Stream(dev) for _ in range(WORLD)]
    import concurrent.futures as cf

    def one(r):
        torch.cuda.set_device(dev)
        with torch.cuda.stream(streams[r]):
            loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True, shard=specs[r])
            opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=int(f["m"]),
                                  tolerance=1e-9, tqdm=False)
            tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=1)
            opt.compute_loss_of_iterates()
            x = opt.x.cpu().numpy()
            out = (list(tr.loss_vals), x)
            loss.device_matrix.close()
            return out

    try:
        with cf.ThreadPoolExecutor(max_workers=WORLD) as ex:
            futs = [ex.submit(one, r) for r in range(WORLD)]
            cf.wait(futs)
        res = [fu.result() for fu in futs]
    finally:
        for c in comms:
            c.close()
    st = int(f["stride"])
    for lv, x in res:
        np.testing.assert_allclose(lv, f["crn_loss_vals"], rtol=1e-10)
        assert rel_err(x[::st], f["crn_final_x_sample"]) < 1e-10
        np.testing.assert_array_equal(x, res[0][1])


def test_rows_x2_unequal_blocks_agree():
    """row shards pack their pass-1 alpha partials past the
    d-vector of the one all-reduce per Lanczos step, and a rank's partial count
    follows its own block.  On a skewed matrix the nnz-balanced split gives
    the two ranks blocks of very different row counts (so different pass-1
    grids); the ranks agree on the packed length at attach time
    (krcn_plan.hip agree_rows), the shorter one zero-fills, and the recurrence
    must still match the oracle at the golden tolerance (alphas / betas 1e-11,
    m = 10; reference cubic.py:77-111 over loss.py:289-302)."""
    import scipy.sparse as sp

    import krcn_oracle as O
    # 2,000 rows of 100 nonzeros, then 10,000 rows of 20: the nnz-balanced
    # split gives rank 0 the first 2,000 rows and rank 1 the other 10,000
    rng = np.random.default_rng(41)
    n, d = 12_000, 30_000
    lens = np.concatenate([np.full(2_000, 100), np.full(10_000, 20)])
    indptr = np.concatenate([[0], np.cumsum(lens)])
    cols = np.concatenate([np.sort(rng.choice(d, k, replace=False)) for k in lens])
    A = sp.csr_matrix((rng.uniform(-1, 1, indptr[-1]), cols.astype(np.int32), indptr.astype(np.int32)), shape=(n, d))
    b = np.where(A @ rng.uniform(-1, 1, d) >= 0, 1.0, -1.0)
    vs = kdist.VirtualShards(A, b, 2, partition="rows")
    try:
        rows = np.diff(vs.bounds)
        assert max(rows) > 3 * min(rows), rows
        m = 10

        def fn(r):
            X = vs.X[r]
            x = torch.full((X.d,), 0.5, dtype=X.dtype, device=X.device)
            Ax = X.matvec(x)
            g = X.gradient(Ax, vs.b[r])
            _, al, be, info = X.lanczos(X.weights(Ax), g, m)
            return al, be, info.m_eff, X.plan_info(), g.cpu().numpy()

        res = vs.run(fn)
    finally:
        vs.close()
    assert res[0][3] != res[1][3]   # the ranks' plans differ
    x = np.full(A.shape[1], 0.5)
    wh = O.hessian_weights(A, x)
    _, al_r, be_r, _ = O.lanczos(lambda v: O.hvp_from_weights(A, wh, v), O.gradient(A, O.labels01(b), x), m)
    for al, be, m_eff, _, _ in res:
        assert m_eff == m
        assert rel_err(al, al_r) < 1e-11
        assert rel_err(be, be_r) < 1e-11
        np.testing.assert_array_equal(al, res[0][0])
