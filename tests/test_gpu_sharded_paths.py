"""Sharded code paths on one GPU.

The ROWS / COLS shard modes route through different kernels (raw partial
passes, elementwise epilogues, scalar all-reduces of the Lanczos dots).  With
a 1-rank RCCL communicator every all-reduce is the identity, so a handle that
holds the whole matrix in a shard mode must reproduce the unsharded results;
this exercises those kernels without a second GPU.  The collective itself is
exercised by the multi-GPU bench (N > 1) and the partition logic by the gloo
tests (tests/test_dist_gloo.py).
"""
import numpy as np
import pytest
import torch

import krcn
import krcn_oracle as O
from conftest import golden_csr, load_golden, rel_err
from krcn import _lib
from krcn.dist import Communicator

pytestmark = pytest.mark.gpu
DEV = "cuda"


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, torch.float64)


@pytest.fixture(scope="module")
def comm():
    c = Communicator(1, 0, torch.device(DEV, 0), Communicator.unique_id())
    yield c
    c.close()


@pytest.mark.parametrize("mode", [_lib.KRCN_SHARD_ROWS, _lib.KRCN_SHARD_COLS])
@pytest.mark.parametrize("slicing", [1, 8])
def test_shard_modes_single_rank(f1, f2, comm, mode, slicing):
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A, shard_mode=mode, slicing=slicing)
    X.attach_comm(comm)
    b01 = t(O.labels01(f1["b"]))
    x = t(f1["x0"])
    Ax = X.matvec(x)
    assert rel_err(Ax.cpu().numpy(), f1["Ax0"]) < 1e-13
    w = X.weights(Ax)
    g = X.gradient(Ax, b01)
    assert rel_err(g.cpu().numpy(), f1["grad0"]) < 1e-13
    assert rel_err(X.hvp(w, t(f1["v0"])).cpu().numpy(), f1["hvp0_0"]) < 1e-13
    assert abs(X.loss_mean(Ax, b01) - f1["value0"]) <= 1e-13 * abs(f1["value0"])
    V, al, be, info = X.lanczos(w, g, 10)
    assert info.m_eff == 10
    assert rel_err(al, f2["alphas_m10"]) < 1e-11
    assert rel_err(be, f2["betas_m10"]) < 1e-11
    assert abs(X.diff_norm(g) - np.linalg.norm(f1["grad0"])) < 1e-13 * np.linalg.norm(f1["grad0"])


@pytest.mark.parametrize("mode", [_lib.KRCN_SHARD_ROWS, _lib.KRCN_SHARD_COLS])
def test_shard_modes_breakdown(f2, comm, mode):
    A = golden_csr(f2, "r3_")
    X = krcn.DeviceCSR(A, shard_mode=mode)
    X.attach_comm(comm)
    x = t(np.full(A.shape[1], 0.5))
    Ax = X.matvec(x)
    g = X.gradient(Ax, t(O.labels01(f2["r3_b"])))
    for m in (4, 5):
        V, al, be, info = X.lanczos(X.weights(Ax), g, m)
        assert info.breakdown and info.j_break == 2
        assert rel_err(al, f2[f"r3_m{m}_alphas"]) < 1e-11
        np.testing.assert_allclose(be, f2[f"r3_m{m}_betas"], rtol=1e-11, atol=0)


@pytest.mark.parametrize("mode", [_lib.KRCN_SHARD_ROWS, _lib.KRCN_SHARD_COLS])
@pytest.mark.parametrize("m", [1, 5, 10])
def test_shard_modes_lanczos_l2(f1, comm, mode, m):
    """l2 = 0.01 through the single-collective early-alpha step of both shard
    modes (alpha formed as (X v).(w X v) / n + l2 - z.v), against
    the oracle's Lanczos over hvp_from_weights(.., l2) at 1e-11."""
    A = golden_csr(f1)
    X = krcn.DeviceCSR(A, shard_mode=mode)
    X.attach_comm(comm)
    x = t(f1["x0"])
    Ax = X.matvec(x)
    w = X.weights(Ax)
    g = X.gradient(Ax, t(O.labels01(f1["b"])))
    V, al, be, info = X.lanczos(w, g, m, l2=0.01)
    wh = O.hessian_weights(A, f1["x0"])
    Vr, al_r, be_r, beta_r = O.lanczos(lambda v: O.hvp_from_weights(A, wh, v, l2=0.01), g.cpu().numpy(), m)
    assert info.m_eff == m
    assert rel_err(al, al_r) < 1e-11
    assert rel_err(be, be_r) < 1e-11
    assert np.abs(V.cpu().numpy()[:m].T - Vr).max() < 1e-6
