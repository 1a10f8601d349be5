"""Binary label mapping of the reference's LogisticRegression (loss.py:189-207).

Shared by the drop-in loss (optimizer/loss.py) and the benchmark / shard
helpers (krcn.dist), so every entry point maps {-1,1}, {1,2}, {0,1} and other
two-valued label sets to {0, 1} the same way.
"""
from __future__ import annotations

import warnings

import numpy as np


def labels01(b):
    """Map binary labels to {0, 1} exactly as loss.py:189-207 does."""
    b = np.asarray(b)
    uniq = np.unique(b)
    if len(uniq) == 1:
        warnings.warn("The labels have only one unique value.")
    if len(uniq) > 2:
        raise ValueError("The number of classes must be no more than 2 for binary classification.")
    if len(uniq) == 2 and (uniq != [0, 1]).any():
        if (uniq == [1, 2]).all():
            return b - 1
        if (uniq == [-1, 1]).all():
            return (b + 1) / 2
        return 1.0 * (b == b[0])
    return b
