"""hipGraph replay of the device Lanczos (krcn_lanczos_impl.hpp, cubic.py:77-111).

An unsharded call records its launch sequence as a graph the second time the
same arguments (w, g, V, m, reorth, tol, l2 and the handle's workspace
generation) arrive and replays it from the third call on.  The replay must be
bitwise the eager launch sequence (replay off) on every plan family the auto
policy picks: fused window slices, fused sorted tiles, the fused one-piece
window (w8a shape), the unfused jagged path and CGS2 reorthogonalisation; and
it must read its operands at run time (new contents behind the same pointers).
Replay is opt-in (krcn_csr_set_graph, DeviceCSR.set_graph); the tests switch it per call.
"""
import numpy as np
import pytest
import torch

import krcn
import krcn_oracle as O
from conftest import golden_csr
from krcn import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def operator(A, b, x, dtype=torch.float64):
    X = krcn.DeviceCSR(A, dtype=dtype)
    Ax = X.matvec(torch.from_numpy(np.ascontiguousarray(x)).to(DEV, dtype))
    w = X.weights(Ax)
    g = X.gradient(Ax, torch.from_numpy(O.labels01(b)).to(DEV, dtype))
    return X, w, g


def run(X, w, g, m, V, reorth=False):
    _, al, be, info = X.lanczos(w, g, m, reorth=reorth, V=V)
    return al, be, V.clone(), info


def check_replay(monkeypatch, X, w, g, m, reorth=False, calls=5):
    V = torch.empty((m, X.d), dtype=X.dtype, device=DEV)
    X.set_graph(False)
    # past the w placement probe (fused window plans, calls 1..4) so W is settled
    for _ in range(calls):
        ref = run(X, w, g, m, V, reorth)
    X.set_graph(True)
    for k in range(3):   # eager (new key) -> record + launch -> replay
        al, be, Vg, info = run(X, w, g, m, V, reorth)
        np.testing.assert_array_equal(al, ref[0], err_msg=f"call {k}")
        np.testing.assert_array_equal(be, ref[1], err_msg=f"call {k}")
        assert torch.equal(Vg, ref[2]), k
        assert (info.m_eff, info.hvps, info.breakdown) == (ref[3].m_eff, ref[3].hvps, ref[3].breakdown)
    return V


@pytest.mark.parametrize("shape", ["rcv1", "w8a", "news20"])
def test_graph_replay_bitwise(monkeypatch, shape):
    kw = {"w8a": dict(n=20_000, nnz=230_000)}.get(shape, {})
    A, b = synth.make_problem(shape, **kw)
    X, w, g = operator(A, b, np.full(A.shape[1], 0.5))
    check_replay(monkeypatch, X, w, g, {"rcv1": 50, "w8a": 10, "news20": 100}[shape])


def test_graph_replay_reorth_fp32(monkeypatch):
    A, b = synth.make_problem("rcv1")
    X, w, g = operator(A, b, np.full(A.shape[1], 0.5), dtype=torch.float32)
    check_replay(monkeypatch, X, w, g, 64, reorth=True, calls=1)


def test_graph_reads_operands_at_run_time(monkeypatch, f1):
    """Same pointers, new contents: the replay follows the new g / w, and a
    new m records a new graph."""
    A = golden_csr(f1)
    X, w, g = operator(A, f1["b"], f1["x0"])
    _, w1, g1 = operator(A, f1["b"], f1["x1"])
    V = check_replay(monkeypatch, X, w, g, 10)
    w.copy_(w1)
    g.copy_(g1)
    al, be, _, _ = run(X, w, g, 10, V)          # replayed
    X.set_graph(False)
    al0, be0, _, _ = run(X, w, g, 10, V)
    np.testing.assert_array_equal(al, al0)
    np.testing.assert_array_equal(be, be0)
    X.set_graph(True)
    V2 = torch.empty((12, X.d), dtype=X.dtype, device=DEV)
    for _ in range(3):
        al, _, _, _ = run(X, w, g, 12, V2)
    X.set_graph(False)
    al0, _, _, _ = run(X, w, g, 12, V2)
    np.testing.assert_array_equal(al, al0)
