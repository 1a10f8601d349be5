"""Multi-process sharding logic on CPU (gloo, world size 2).

The HIP path shards X by rows or columns (krcn.dist) and all-reduces inside
the recurrence.  Here every rank runs the oracle's arithmetic on its own block
(krcn.dist.plan / extract) and exchanges partials with gloo all-reduces at the
same points the device path calls RCCL; the result must equal the unsharded
oracle.  This pins the partition and the decomposition; the kernels are
covered by tests/test_gpu_sharded_paths.py.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import krcn_oracle as O
from krcn import dist as kd
from krcn import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _allreduce(a):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
    dist.all_reduce(t)
    return t.numpy()


def _lanczos_rows(Ap, wp, g, m, n, l2):
    """The row-shard recurrence as the device runs it (krcn_lanczos_impl.hpp
    early_rows): d-vectors replicated, ONE all-reduce per step carrying the
    d-length X_p^T u_p with this rank's alpha partial (X v).(w X v) packed past
    element d; beta and z.v_{j-1} are d-space sums, the same on every rank."""
    zz, zv = float(g @ g), 0.0
    z, vp = g, np.zeros_like(g)
    al, be = [], []
    nrm = np.sqrt(zz)
    for j in range(m - 1):
        if j > 0:
            nrm = np.sqrt(zz)
            be.append(nrm)
        q = (Ap @ z) / nrm                              # pass 1 + combine: q = t / beta
        u = wp * q
        buf = _allreduce(np.concatenate([Ap.T @ u, [u @ q]]))
        a = buf[-1] / n + l2 - zv                       # early alpha (z_j . v_{j-1} = beta v_j . v_{j-1})
        v = z / nrm
        y = buf[:-1] / n + l2 * v
        wv = y - (be[-1] * vp if j > 0 else 0.0)
        z, vp = wv - a * v, v
        zz, zv = float(z @ z), float(z @ v)
        al.append(a)
    nrm = np.sqrt(zz)
    be.append(nrm)
    v = z / nrm
    y = _allreduce(Ap.T @ (wp * ((Ap @ z) / nrm))) / n + l2 * v
    al.append(float(v @ y))                              # the final quotient (cubic.py:109)
    return np.array(al), np.array(be)


def _lanczos_cols(Ap, w, g, m, n, l2):
    """The column-shard recurrence as the device runs it (early_cols): the
    d-vectors are sharded, and each step has ONE all-reduce of n + 2 values:
    X_p z_p with this rank's ||z_p||^2 and z_p . v_{p,j-1} packed as elements
    n and n + 1 (step 0: n values, ||g||^2 was all-reduced at the start); the
    row apply then settles beta and u = w (t / beta) replicated over n, so the
    alpha of pass 2 needs no collective of its own.  The last step's norm and
    the final quotient take scalar all-reduces (k_lz_final_check, k_lz_final)."""
    ar = _allreduce
    nrm = np.sqrt(ar([g @ g])[0])
    z, vp = g, np.zeros_like(g)
    zz = zv = 0.0
    al, be = [], []
    for j in range(m - 1):
        t = Ap @ z
        if j == 0:
            buf = ar(t)
            zvg = 0.0
        else:
            buf = ar(np.concatenate([t, [zz, zv]]))
            nrm, zvg = np.sqrt(buf[n]), buf[n + 1]
            be.append(nrm)
        q = buf[:n] / nrm
        u = w * q
        a = (u @ q) / n + l2 - zvg
        v = z / nrm
        y = Ap.T @ u / n + l2 * v
        wv = y - (be[-1] * vp if j > 0 else 0.0)
        z, vp = wv - a * v, v
        zz, zv = float(z @ z), float(z @ v)
        al.append(a)
    nrm = np.sqrt(ar([zz])[0])
    be.append(nrm)
    v = z / nrm
    y = Ap.T @ (w * (ar(Ap @ z) / nrm)) / n + l2 * v
    al.append(float(ar([v @ y])[0]))
    return np.array(al), np.array(be)


def _worker(rank, world, port, mode, l2, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A, b = synth.make_problem(None, seed=11, n=300, d=700, nnz=6000)
    n, d = A.shape
    b01 = O.labels01(b)
    x = np.linspace(-0.3, 0.3, d)
    mode_, bounds = kd.plan(A, world, mode)
    Ap = kd.extract(A, mode_, bounds, rank)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    rng = np.random.default_rng(5)
    v = rng.standard_normal(d)
    m = 8
    if mode_ == "rows":
        Axp = Ap @ x                                   # local rows
        wp = O.hessian_weights(Ap, x)
        y = _allreduce(Ap.T @ (wp * (Ap @ v))) / n     # d-length all-reduce
        g = _allreduce(Ap.T @ (1 / (1 + np.exp(-Axp)) - b01[lo:hi])) / n
        al, be = _lanczos_rows(Ap, wp, g, m, n, l2)
    else:
        t = _allreduce(Ap @ x[lo:hi])                  # n-length all-reduce of X_p x_p
        w = 1 / (1 + np.exp(-t))
        w = w * (1 - w)
        y = (Ap.T @ (w * _allreduce(Ap @ v[lo:hi]))) / n
        g = Ap.T @ (1 / (1 + np.exp(-t)) - b01) / n
        al, be = _lanczos_cols(Ap, w, g, m, n, l2)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), y=y, g=g, lo=lo, hi=hi, al=al, be=be, mode=np.array(mode_))
    dist.destroy_process_group()


@pytest.mark.parametrize("l2", [0.0, 0.01])
@pytest.mark.parametrize("mode", ["rows", "cols"])
def test_two_rank_shards_match_unsharded(mode, l2):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(2, _free_port(), mode, l2, td), nprocs=2, join=True)
        r = [np.load(os.path.join(td, f"r{k}.npz")) for k in range(2)]
    A, b = synth.make_problem(None, seed=11, n=300, d=700, nnz=6000)
    x = np.linspace(-0.3, 0.3, A.shape[1])
    v = np.random.default_rng(5).standard_normal(A.shape[1])
    y_ref = O.hess_vec_prod(A, x, v)
    g_ref = O.gradient(A, O.labels01(b), x)
    w = O.hessian_weights(A, x)
    _, al_ref, be_ref, _ = O.lanczos(lambda q: O.hvp_from_weights(A, w, q, l2=l2), g_ref, 8)
    if mode == "rows":
        for k in range(2):       # d-vectors replicated after the all-reduce
            np.testing.assert_allclose(r[k]["y"], y_ref, rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(r[k]["g"], g_ref, rtol=1e-12, atol=1e-15)
    else:                        # d-vectors sharded: concatenate the column blocks
        y = np.concatenate([r[k]["y"] for k in range(2)])
        g = np.concatenate([r[k]["g"] for k in range(2)])
        assert int(r[0]["hi"]) == int(r[1]["lo"])
        np.testing.assert_allclose(y, y_ref, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(g, g_ref, rtol=1e-12, atol=1e-15)
    for k in range(2):
        np.testing.assert_allclose(r[k]["al"], al_ref, rtol=1e-10)
        np.testing.assert_allclose(r[k]["be"], be_ref, rtol=1e-10)
        np.testing.assert_array_equal(r[k]["al"], r[0]["al"])   # the scalars are the same on every rank


def test_plan_balances_and_covers():
    A, _ = synth.make_problem("rcv1", skew=True)
    for world in (2, 4, 8):
        for mode in ("rows", "cols"):
            m, bounds = kd.plan(A, world, mode)
            assert m == mode and bounds[0] == 0
            assert bounds[-1] == (A.shape[0] if mode == "rows" else A.shape[1])
            assert np.all(np.diff(bounds) >= 0)
            parts = [kd.extract(A, m, bounds, r).nnz for r in range(world)]
            assert sum(parts) == A.nnz
            assert max(parts) <= 1.25 * A.nnz / world + 20000   # nnz-balanced up to one hot column
    assert kd.choose_partition(19996, 1355191, 8) == "cols"
    assert kd.choose_partition(2_000_000, 1_000_000, 8) == "rows"
    assert kd.choose_partition(100, 200, 1) == "none"


def test_plan_dominant_column_leaves_no_rank_empty():
    """One dense column (a bias feature) holding most of the nonzeros must not
    leave a rank with an empty column range: that rank would skip the RCCL
    all-reduces its peers block in (krcn/dist.py balanced_ranges)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(3)
    n, d = 4000, 64
    rows = np.concatenate([np.arange(n), rng.integers(0, n, 600)])
    cols = np.concatenate([np.zeros(n, dtype=np.int64), rng.integers(1, d, 600)])
    A = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(n, d))
    for world in (2, 4, 8):
        _, bounds = kd.plan(A, world, "cols")
        assert bounds[0] == 0 and bounds[-1] == d
        assert np.all(np.diff(bounds) >= 1), bounds
        assert sum(kd.extract(A, "cols", bounds, r).nnz for r in range(world)) == A.nnz
    # fewer columns than ranks cannot give every rank one: the cuts stay monotone
    b = kd.balanced_ranges([5, 1], 4)
    assert b[0] == 0 and b[-1] == 2 and np.all(np.diff(b) >= 0)
    with pytest.raises(ValueError, match="empty block"):
        kd.plan(A[:, :3], 4, "cols")
