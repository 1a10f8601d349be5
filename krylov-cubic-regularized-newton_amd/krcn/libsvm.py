"""LIBSVM / svmlight datasets from a local file.

The reference downloads a LIBSVM binary-classification dataset
(urllib.request.urlretrieve, cubic_newton.py:43-51) and reads it with
sklearn.datasets.load_svmlight_file (cubic_newton.py:52-53), a single-threaded
Cython line loop.  There is no network here, so `load` takes a local path.

The default parser is libkrcn's native one (krcn_svm_parse,
csrc/krcn_svmlight.hip): the text is cut into byte ranges at line boundaries
and parsed by one thread each, then stitched into one CSR.  Its result is
sklearn's, array for array and bit for bit (tests/test_libsvm.py):
  * the same grammar (comments, blank lines, a leading qid:, signed labels /
    indices, correctly rounded decimal floats, inf / nan);
  * the same errors: a negative index, index 0 in a one-based file, and
    indices that are not strictly increasing within a row (sklearn rejects
    duplicates rather than summing them);
  * zero_based="auto": one-based (indices shifted down by one) unless some
    index is 0; n_features = the largest index + 1 unless given;
  * CSR float64 (or float32 via dtype) with int32 indices and row pointers,
    labels float64.
`parser="sklearn"` keeps the reference's own loader.  `load_device` uploads
the matrix once as a DeviceCSR (the transpose and the pass plans are built on
the GPU); krcn.dist.plan cuts it for a sharded run.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import scipy.sparse as sp


def _read_text(path):
    if path.endswith(".gz"):
        import gzip
        with gzip.open(path, "rb") as f:
            return f.read()
    if path.endswith(".bz2"):
        import bz2
        with bz2.open(path, "rb") as f:
            return f.read()
    with open(path, "rb") as f:
        return f.read()


def parse(text, n_features=None, zero_based="auto", dtype=np.float64, threads=None):
    """(A, b) from svmlight text (bytes) with the native parser."""
    from . import _lib
    if isinstance(text, str):
        text = text.encode()
    threads = threads or min(16, len(os.sched_getaffinity(0)))
    lib = _lib.load()
    h = ctypes.c_void_p()
    info = (ctypes.c_int64 * 4)()
    buf = ctypes.c_char_p(text)
    st = lib.krcn_svm_parse(buf, len(text), int(threads), ctypes.byref(h), info)
    if st != _lib.KRCN_OK:
        raise ValueError(lib.krcn_last_error_string().decode())
    try:
        n, nnz, max_index, min_index = (int(v) for v in info)
        if zero_based is False and nnz and min_index == 0:
            raise ValueError("Invalid index 0 in SVMlight/LibSVM data file.")
        # sklearn: one-based unless some index is 0 (auto), or told so
        shift = 1 if (zero_based is False or (zero_based == "auto" and nnz and min_index > 0)) else 0
        n_f = (max_index - shift if nnz else 0) + 1
        if n_features is None:
            n_features = n_f
        elif n_features < n_f:
            raise ValueError(f"n_features was set to {n_features}, but input file contains {n_f} features")
        indptr = np.empty(n + 1, dtype=np.int32)
        indices = np.empty(nnz, dtype=np.int32)
        data = np.empty(nnz, dtype=np.float64)
        labels = np.empty(n, dtype=np.float64)
        _lib.call("krcn_svm_export", h, shift, indptr.ctypes.data_as(ctypes.c_void_p),
                  indices.ctypes.data_as(ctypes.c_void_p), data.ctypes.data_as(ctypes.c_void_p),
                  labels.ctypes.data_as(ctypes.c_void_p))
    finally:
        lib.krcn_svm_destroy(h)
    if np.dtype(dtype) != np.float64:
        with np.errstate(over="ignore"):   # as sklearn's C float cast: out of range -> inf
            data = data.astype(dtype)
    A = sp.csr_matrix((data, indices, indptr), shape=(n, int(n_features)))
    return A, labels


def load(path, n_features=None, zero_based="auto", dtype=np.float64, parser="native", threads=None):
    """(A, b) from a LIBSVM / svmlight text file (optionally .gz / .bz2)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path}: no such dataset (datasets are not downloaded here)")
    if parser == "sklearn":
        from sklearn.datasets import load_svmlight_file
        A, b = load_svmlight_file(path, n_features=n_features, zero_based=zero_based, dtype=dtype)
        A = sp.csr_matrix(A, dtype=dtype)
    elif parser == "native":
        A, b = parse(_read_text(path), n_features=n_features, zero_based=zero_based, dtype=dtype,
                     threads=threads)
    else:
        raise ValueError(f"parser must be 'native' or 'sklearn', got {parser!r}")
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
