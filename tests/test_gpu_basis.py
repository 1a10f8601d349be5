"""x + V^T s (cubic.py:291, krcn_basis_combine) against the sequential numpy
sum in j order: bitwise in fp64 (the kernel adds its batched row loads in the
same order, no contraction), for m on both sides of the 16-row load batch."""
import numpy as np
import pytest
import torch

import krcn
from krcn import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m", [1, 15, 16, 17, 100])
def test_basis_combine_bitwise(m):
    A, _ = synth.make_problem(None, seed=7, n=300, d=5003, nnz=9000)
    X = krcn.DeviceCSR(A)
    rng = np.random.default_rng(m)
    V = rng.standard_normal((m, X.d))
    s = rng.standard_normal(m)
    x = rng.standard_normal(X.d)
    acc = np.zeros(X.d)
    for j in range(m):
        acc = acc + V[j] * s[j]
    ref = x + acc
    # the Lanczos workspace bounds m: size it with one call first
    w = torch.ones(X.n, dtype=torch.float64, device="cuda")
    X.lanczos(w, torch.ones(X.d, dtype=torch.float64, device="cuda"), max(m, 2))
    out = X.basis_combine(torch.from_numpy(V).cuda(), s, torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
