"""Test configuration.

Markers: `gpu` tests need an MI355X (they run through libkrcn.so's C ABI and
are the parity tests proper); everything else runs on CPU in the build
container (oracle vs golden vectors, host logic, ABI loading, gloo sharding).
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "krylov-cubic-regularized-newton_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs the HIP path)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_csr(f, prefix=""):
    import scipy.sparse as sp
    shape = tuple(int(s) for s in f[f"{prefix}shape"])
    return sp.csr_matrix((f[f"{prefix}data"], f[f"{prefix}indices"], f[f"{prefix}indptr"]), shape=shape)


@pytest.fixture(scope="session")
def f1():
    return load_golden("f1_hvp.npz")


@pytest.fixture(scope="session")
def f2():
    return load_golden("f2_lanczos.npz")


@pytest.fixture(scope="session")
def f3():
    return load_golden("f3_cubic.npz")


@pytest.fixture(scope="session")
def f4():
    return load_golden("f4_traj.npz")


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max() if b.size else 0.0, 1e-300)
    return float(np.abs(a - b).max() / scale) if a.size else 0.0
