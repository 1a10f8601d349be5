"""Host glue shared by the drop-in modules (mirrors optimizer/utils.py of the
reference: safe_sparse_add / inner_prod / multiply / norm, utils.py:11-62).

They accept numpy arrays, scipy.sparse matrices and (for the device path) torch
tensors; device tensors never leave the GPU here.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

try:
    import torch
except ImportError:  # pragma: no cover - torch is a hard dependency of the device path
    torch = None


def _is_tensor(a):
    return torch is not None and isinstance(a, torch.Tensor)


def safe_sparse_add(a, b):
    """a + b for scalars, dense arrays and sparse matrices (utils.py:11-33):
    sparse + sparse stays sparse, anything mixed becomes dense."""
    if (sp.issparse(a) and sp.issparse(b)) or np.isscalar(a) or np.isscalar(b):
        return a + b
    if sp.issparse(a):
        a = a.toarray()
        if a.ndim == 2 and np.ndim(b) == 1:
            a = a.ravel()
    if sp.issparse(b):
        b = b.toarray()
        if b.ndim == 2 and np.ndim(a) == 1:
            b = b.ravel()
    return a + b


def safe_sparse_inner_prod(a, b):
    """<a, b> for dense / sparse vectors (utils.py:35-47)."""
    if sp.issparse(a) and sp.issparse(b):
        if a.ndim == 2 and a.shape[1] == b.shape[0]:
            return (a @ b)[0, 0]
        if a.shape[0] == b.shape[0]:
            return (a.T @ b)[0, 0]
        return (a @ b.T)[0, 0]
    if sp.issparse(a):
        a = a.toarray()
    elif sp.issparse(b):
        b = b.toarray()
    return a @ b


def safe_sparse_multiply(a, b):
    """Elementwise a * b (utils.py:49-58)."""
    if sp.issparse(a):
        return a.multiply(b)
    if sp.issparse(b):
        b = b.toarray()
    return np.multiply(a, b)


def safe_sparse_norm(a, ord=None):
    """||a|| for dense or sparse input (utils.py:60-62)."""
    if sp.issparse(a):
        return sp.linalg.norm(a, ord=ord)
    return np.linalg.norm(a, ord=ord)
