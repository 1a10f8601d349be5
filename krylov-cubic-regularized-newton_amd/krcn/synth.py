"""Deterministic synthetic LIBSVM-shaped logistic-regression problems.

There are no LIBSVM files on the build or GPU machines (the reference downloads
them, cubic_newton.py:43-51), so every configuration of BASELINE.json runs on a
shape-matched synthetic CSR matrix.  The generator is counter-based (splitmix64
of a per-stream key plus the element index), written with numpy uint64
arithmetic only, so any machine regenerates the same matrix bit for bit from
(config, seed) — golden statistics computed here by the reference are valid on
the GPU box.

Shapes (dataset pages cited by cubic_newton.py:43):
  w8a    n 49,749     d 300        nnz 580,000      binary values
  rcv1   n 20,242     d 47,236     nnz 1,498,952    U(-1,1)
  news20 n 19,996     d 1,355,191  nnz 9,097,916    U(-1,1)
  synth  n 2,000,000  d 1,000,000  nnz 200,000,000  U(-1,1)
Uniform variant: equal row lengths (±1), one column per equal-width stratum of
[0, d) per row (sorted, unique, marginally uniform).  Skewed variant: lognormal
row lengths and power-law column popularity (hot columns scattered by a
multiplicative hash), deduplicated per row.
Labels are ±1 from a planted model, b = sign(X x* + 0.1 e).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

SEED = 20240117

CONFIGS = {
    "w8a": dict(n=49_749, d=300, nnz=580_000, values="binary", m=10, dtype="f64"),
    "rcv1": dict(n=20_242, d=47_236, nnz=1_498_952, values="uniform", m=50, dtype="f64"),
    "news20": dict(n=19_996, d=1_355_191, nnz=9_097_916, values="uniform", m=100, dtype="f64"),
    "rcv1_stress": dict(n=20_242, d=47_236, nnz=1_498_952, values="uniform", m=500, dtype="f32",
                        reorth=True),
    "synth": dict(n=2_000_000, d=1_000_000, nnz=200_000_000, values="uniform", m=50, dtype="f64"),
}

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _stream_key(seed: int, stream: int) -> np.uint64:
    with np.errstate(over="ignore"):
        k = _splitmix64(np.array([(seed * 0x100000001B3 + stream) & 0xFFFFFFFFFFFFFFFF],
                                 dtype=np.uint64))
    return k[0]


def uniform01(seed: int, stream: int, count: int, offset: int = 0) -> np.ndarray:
    """count doubles in [0, 1): top 53 bits of splitmix64(key + i) * 2^-53."""
    key = _stream_key(seed, stream)
    with np.errstate(over="ignore"):
        c = np.arange(offset, offset + count, dtype=np.uint64) + key
        u = _splitmix64(c)
    return (u >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _uniform_pattern(n, d, nnz, seed):
    base, rem = divmod(nnz, n)
    lengths = np.full(n, base, dtype=np.int64)
    lengths[:rem] += 1
    lengths = np.minimum(lengths, d)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lengths, out=indptr[1:])
    total = int(indptr[-1])
    row = np.repeat(np.arange(n, dtype=np.int64), lengths)
    k = np.arange(total, dtype=np.int64) - indptr[row]
    L = lengths[row]
    lo = (k * d) // L
    hi = ((k + 1) * d) // L
    del row, k, L
    u = uniform01(seed, 1, total)
    cols = lo + np.minimum((u * (hi - lo)).astype(np.int64), hi - lo - 1)
    return indptr, cols


def _skewed_pattern(n, d, nnz, seed, sigma=1.0, gamma=3.0):
    z = uniform01(seed, 11, n)
    z2 = uniform01(seed, 12, n)
    # Box-Muller normal -> lognormal row lengths scaled to ~nnz
    g = np.sqrt(-2.0 * np.log(np.maximum(z, 1e-300))) * np.cos(2.0 * np.pi * z2)
    raw = np.exp(sigma * g)
    lengths = np.clip(np.floor(raw * (nnz / raw.sum())), 1, d).astype(np.int64)
    row = np.repeat(np.arange(n, dtype=np.int64), lengths)
    total = row.size
    u = uniform01(seed, 13, total)
    rank = np.minimum((d * u ** gamma).astype(np.int64), d - 1)
    mult = 2654435761 % d or 1
    while np.gcd(mult, d) != 1:
        mult += 1
    cols = (rank * mult) % d
    key = np.unique(row * d + cols)
    row = key // d
    cols = key % d
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(row, minlength=n), out=indptr[1:])
    return indptr, cols


def make_problem(config="news20", seed=SEED, skew=False, n=None, d=None, nnz=None,
                 values=None):
    """Return (A, b): A scipy CSR float64 (int32 indices), b float64 labels in {-1, +1}."""
    cfg = dict(CONFIGS[config]) if config is not None else {}
    n = int(n if n is not None else cfg["n"])
    d = int(d if d is not None else cfg["d"])
    nnz = int(nnz if nnz is not None else cfg["nnz"])
    values = values or cfg.get("values", "uniform")
    if skew:
        indptr, cols = _skewed_pattern(n, d, nnz, seed)
    else:
        indptr, cols = _uniform_pattern(n, d, nnz, seed)
    total = int(indptr[-1])
    if values == "binary":
        data = np.ones(total, dtype=np.float64)
    else:
        data = 2.0 * uniform01(seed, 2, total) - 1.0
    A = sp.csr_matrix((data, cols.astype(np.int32), indptr.astype(np.int32)), shape=(n, d))
    xstar = 2.0 * uniform01(seed, 3, d) - 1.0
    noise = 2.0 * uniform01(seed, 4, n) - 1.0
    margin = A @ xstar + 0.1 * noise
    b = np.where(margin >= 0.0, 1.0, -1.0)
    return A, b


def hvp_bytes(n, d, nnz, s_val=8, s_idx=4, s_ptr=4):
    """Algorithmic bytes of one HVP:
    2 nnz (s_val + s_idx) + s_ptr ((n+1) + (d+1)) + s_val (2d + 3n)."""
    return 2 * nnz * (s_val + s_idx) + s_ptr * ((n + 1) + (d + 1)) + s_val * (2 * d + 3 * n)


def pass_bytes(n, d, nnz, s_val=8, s_idx=4, s_ptr=4):
    """Split of hvp_bytes over the two launches: pass 1 reads X, v (d), w and
    writes u; pass 2 reads X^T, u and writes y."""
    p1 = nnz * (s_val + s_idx) + s_ptr * (n + 1) + s_val * (d + 2 * n)
    p2 = nnz * (s_val + s_idx) + s_ptr * (d + 1) + s_val * (d + n)
    return p1, p2


def lanczos_pass_bytes(n, d, nnz, s_val=8, s_idx=4, s_ptr=4):
    """Algorithmic bytes of the two launches of one device Lanczos step
    (pass 1: X z + weights; pass 2: X^T u fused with step A, which reads z and
    v_pre and writes v and w instead of writing y)."""
    p1 = nnz * (s_val + s_idx) + s_ptr * (n + 1) + s_val * (d + 2 * n)
    p2 = nnz * (s_val + s_idx) + s_ptr * (d + 1) + s_val * (n + 4 * d)
    return p1, p2


def lanczos_kernel_bytes(n, d, nnz, fused, s_val=8, s_idx=4, s_ptr=4, z_store=False):
    """Algorithmic bytes of each launch of one device Lanczos step (SURVEY.md
    §8d accounting: every stream counted once, index compression and
    implementation partials not counted):
      pass1   X z: X (values + indices + row pointers) and the gathered z (d);
              fused with the previous step B (z = w - alpha v formed from w and
              v in the window: 2 d read; + d written with z_store) when `fused`
      combine u = w (t / beta): w read, u written (n)
      pass2   X^T u fused with step A: X^T, u; w (or z) and v_pre read, v and w
              written (d)
      stepb   z = w - alpha v: w, v read, z written (d) — a launch of its own
              only when not fused."""
    mat = nnz * (s_val + s_idx)
    # fused: the window is z = w - alpha v built from w and v (2 d read); the
    # window-slices pass stores no z (pass 2 re-forms it from w and v_prev,
    # which it reads anyway), the sorted / one-piece fused passes store it
    # (z_store: + d written)
    p1 = mat + s_ptr * (n + 1) + s_val * ((3 if z_store else 2) * d if fused else d)
    return {"pass1": p1, "combine": s_val * 2 * n,
            "pass2": mat + s_ptr * (d + 1) + s_val * (n + 4 * d),
            "stepb": 0 if fused else s_val * 3 * d}
