"""LIBSVM / svmlight datasets from a local file.

The reference downloads a LIBSVM binary-classification dataset
(urllib.request.urlretrieve, cubic_newton.py:43-51) and reads it with
sklearn.datasets.load_svmlight_file (cubic_newton.py:53).  There is no network
here, so `load` takes a local path and reads it with the same sklearn parser,
returning what the reference's LogisticRegression receives: a CSR float64
matrix (int32 indices, sorted, duplicates summed by scipy) and the raw label
vector (LogisticRegression maps it to {0, 1}, loss.py:189-207).
`load_device` uploads the matrix once as a DeviceCSR (the transposed copy and
the pass plans are built on the GPU).
"""
from __future__ import annotations

import os

import numpy as np
import scipy.sparse as sp


def load(path, n_features=None, zero_based="auto", dtype=np.float64):
    """(A, b) from a LIBSVM / svmlight text file (optionally .gz / .bz2)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path}: no such dataset (datasets are not downloaded here)")
    from sklearn.datasets import load_svmlight_file
    A, b = load_svmlight_file(path, n_features=n_features, zero_based=zero_based, dtype=dtype)
    A = sp.csr_matrix(A, dtype=dtype)
    A.sum_duplicates()
    A.sort_indices()
    if A.nnz >= 2 ** 31:
        raise ValueError("more than 2^31 - 1 nonzeros: the device CSR uses int32 offsets")
    A.indices = A.indices.astype(np.int32, copy=False)
    A.indptr = A.indptr.astype(np.int32, copy=False)
    return A, np.asarray(b, dtype=np.float64)


def load_device(path, device=None, dtype=None, **kw):
    """(DeviceCSR, A, b): the file's matrix uploaded once to the GPU."""
    import torch

    from .device import DeviceCSR
    A, b = load(path, **kw)
    X = DeviceCSR(A, device=device, dtype=dtype if dtype is not None else torch.float64)
    return X, A, b
