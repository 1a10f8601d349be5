"""ctypes loader of oracle/krcn_hvp_omp.c -- TEST INFRASTRUCTURE ONLY (tests/,
bench.py's cpu_baseline).  The multi-core C restatement of loss.py:289-302."""
import ctypes
import os

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libkrcn_hvp_omp.so")
_lib = None


def build():
    import subprocess
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-fopenmp", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(HERE, "krcn_hvp_omp.c"), "-o", SO], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            raise FileNotFoundError(f"{SO}: run __graft_entry__.build() first")
        _lib = ctypes.CDLL(SO)
        _lib.krcn_oracle_hvp_omp.restype = ctypes.c_int
    return _lib


class HVP:
    """y = X^T (w * X v) / n + l2 v on `threads` host cores; the transpose is
    built once (scipy tocsc, i.e. rows of X^T sorted)."""

    def __init__(self, A, threads=0):
        A = sp.csr_matrix(A)
        self.n, self.d = A.shape
        self.A = A
        T = A.tocsc()
        self.T = (T.indptr.astype(np.int32), T.indices.astype(np.int32), np.ascontiguousarray(T.data, np.float64))
        self.X = (A.indptr.astype(np.int32), A.indices.astype(np.int32), np.ascontiguousarray(A.data, np.float64))
        self.u = np.empty(self.n)
        self.threads = int(threads)

    def __call__(self, w, v, l2=0.0):
        w = np.ascontiguousarray(w, np.float64)
        v = np.ascontiguousarray(v, np.float64)
        y = np.empty(self.d)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        rc = load().krcn_oracle_hvp_omp(
            ctypes.c_int64(self.n), ctypes.c_int64(self.d), p(self.X[0]), p(self.X[1]), p(self.X[2]),
            p(self.T[0]), p(self.T[1]), p(self.T[2]), p(w), p(v), ctypes.c_double(l2), p(self.u), p(y),
            ctypes.c_int(self.threads))
        if rc:
            raise RuntimeError(f"krcn_oracle_hvp_omp -> {rc}")
        return y
