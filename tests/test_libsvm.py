"""LIBSVM loader (krcn.libsvm): a local svmlight file
reads into the CSR / labels the reference's LogisticRegression receives
(cubic_newton.py:53 uses sklearn's load_svmlight_file on the downloaded file)."""
import numpy as np
import pytest
import scipy.sparse as sp

from krcn import libsvm, synth


def test_round_trip(tmp_path):
    from sklearn.datasets import dump_svmlight_file
    A, b = synth.make_problem(None, seed=5, n=300, d=1000, nnz=6000)
    path = tmp_path / "small.svm"
    dump_svmlight_file(A, b, str(path), zero_based=False)
    A2, b2 = libsvm.load(str(path), n_features=A.shape[1])
    assert A2.indices.dtype == np.int32 and A2.indptr.dtype == np.int32
    assert A2.has_sorted_indices
    np.testing.assert_array_equal(b2, b)
    # dump_svmlight_file writes %.16g: equal to ~1 ulp, same sparsity pattern
    np.testing.assert_array_equal(A2.indptr, A.indptr)
    np.testing.assert_array_equal(A2.indices, A.indices)
    np.testing.assert_allclose(A2.data, A.data, rtol=1e-15, atol=0)
    assert A2.shape == A.shape


def test_text_format_and_labels(tmp_path):
    # 1-based indices as the LIBSVM site ships them, {-1, +1} labels, an empty row
    path = tmp_path / "tiny.svm"
    path.write_text("+1 1:0.5 3:2\n-1 2:1.25\n-1\n+1 3:-1 4:4\n")
    A, b = libsvm.load(str(path), zero_based=False)
    assert A.shape == (4, 4)
    np.testing.assert_array_equal(b, [1, -1, -1, 1])
    np.testing.assert_array_equal(A.toarray(), [[0.5, 0, 2, 0], [0, 1.25, 0, 0], [0, 0, 0, 0], [0, 0, -1, 4]])
    from optimizer.loss import _labels01
    np.testing.assert_array_equal(_labels01(b), [1, 0, 0, 1])


def test_missing_file():
    with pytest.raises(FileNotFoundError):
        libsvm.load("/nonexistent/news20.binary")


def test_matches_scipy_csr(tmp_path):
    from sklearn.datasets import dump_svmlight_file
    rng = np.random.default_rng(0)
    A = sp.random(50, 80, density=0.1, format="csr", random_state=1)
    b = np.where(rng.uniform(size=50) < 0.5, -1.0, 1.0)
    path = tmp_path / "r.svm"
    dump_svmlight_file(A, b, str(path), zero_based=True)
    A2, _ = libsvm.load(str(path), n_features=80, zero_based=True)
    np.testing.assert_allclose(A2.toarray(), A.toarray(), rtol=1e-15, atol=0)


@pytest.mark.gpu
def test_load_device_hvp(tmp_path):
    """A file read through krcn.libsvm runs through the device HVP and matches
    the oracle on the matrix sklearn parsed."""
    import torch
    from sklearn.datasets import dump_svmlight_file

    import krcn_oracle as O
    from conftest import rel_err
    A, b = synth.make_problem(None, seed=8, n=3000, d=60_000, nnz=90_000)
    path = tmp_path / "dev.svm"
    dump_svmlight_file(A, b, str(path), zero_based=False)
    X, A2, b2 = libsvm.load_device(str(path), device="cuda")
    assert X.n == A2.shape[0] and X.nnz == A2.nnz
    x = np.random.default_rng(1).uniform(-0.2, 0.2, size=A2.shape[1])
    v = np.random.default_rng(2).standard_normal(A2.shape[1])
    w = O.hessian_weights(A2, x)
    tt = lambda a: torch.from_numpy(a).to("cuda", torch.float64)
    y = X.hvp(tt(w), tt(v)).cpu().numpy()
    assert rel_err(y, O.hvp_from_weights(A2, w, v)) < 1e-13
    X.close()


# ------------------------------------------------- native parser vs sklearn
def _sk(path, **kw):
    from sklearn.datasets import load_svmlight_file
    return load_svmlight_file(str(path), **kw)


def _same(path, **kw):
    """The native parser's CSR / labels are sklearn's, bit for bit."""
    A, b = libsvm.load(str(path), **kw)
    As, bs = _sk(path, **kw)
    assert A.shape == As.shape and A.dtype == As.dtype
    np.testing.assert_array_equal(A.indptr, As.indptr)
    np.testing.assert_array_equal(A.indices, As.indices)
    assert A.data.tobytes() == As.data.tobytes()
    assert b.tobytes() == np.asarray(bs, dtype=np.float64).tobytes()
    return A, b


def test_native_grammar_matches_sklearn(tmp_path):
    """Comments, blank lines, CRLF, a leading qid, signs, exponents, inf / nan,
    label-only rows, leading / trailing blanks, no final newline."""
    text = ("# header comment\n"
            "+1 qid:7 1:0.5 3:2e0 10:-1.5E-3   # trailing comment\r\n"
            "\n"
            "   -1\t2:.25 4:+7. 5:1e-320\n"
            "0.5\n"
            "-1 1:inf 2:-Infinity 3:nan 6:123456789.123456789123\n"
            "  # only a comment\n"
            "2 7:1e308 8:1e400 9:-1e-400")
    path = tmp_path / "g.svm"
    path.write_bytes(text.encode())
    for zb in ("auto", False, True):
        _same(path, zero_based=zb)
    _same(path, n_features=20)
    _same(path, dtype=np.float32)


def test_native_zero_based_detection(tmp_path):
    p0 = tmp_path / "z.svm"
    p0.write_text("1 0:1 2:2\n-1 5:3\n")
    A, _ = _same(p0)                      # an index 0: zero-based, no shift
    assert A.shape == (2, 6)
    with pytest.raises(ValueError, match="Invalid index 0"):
        libsvm.load(str(p0), zero_based=False)
    p1 = tmp_path / "o.svm"
    p1.write_text("1 1:1 3:2\n-1 5:3\n")
    A, _ = _same(p1)                      # all >= 1: one-based, shifted
    assert A.shape == (2, 5)
    pe = tmp_path / "e.svm"
    pe.write_text("1\n-1\n")
    A, _ = _same(pe)                      # no features at all: one column
    assert A.shape == (2, 1) and A.nnz == 0


@pytest.mark.parametrize("line,msg", [
    ("1 3:1 2:1", "sorted and unique"),
    ("1 2:1 2:1", "sorted and unique"),
    ("1 -2:1", "Invalid index"),
    ("1 2:abc", "could not convert"),
    ("abc 2:1", "could not convert"),
    ("1 x:1", "invalid literal"),
])
def test_native_errors_like_sklearn(tmp_path, line, msg):
    p = tmp_path / "bad.svm"
    p.write_text("1 1:1\n" + line + "\n")
    with pytest.raises(ValueError):
        _sk(p)
    with pytest.raises(ValueError, match=msg):
        libsvm.load(str(p))


def test_native_multithreaded_large_file(tmp_path):
    """A multi-megabyte file (parsed in many byte ranges) equals sklearn's
    result, and the thread count does not change a bit."""
    from sklearn.datasets import dump_svmlight_file
    A, b = synth.make_problem(None, seed=11, n=4000, d=50_000, nnz=300_000)
    path = tmp_path / "big.svm"
    dump_svmlight_file(A, b, str(path), zero_based=False)
    assert path.stat().st_size > (2 << 20)
    A1, b1 = _same(path)
    A2, b2 = libsvm.load(str(path), threads=1)
    A3, b3 = libsvm.load(str(path), threads=13)
    for Ak, bk in ((A2, b2), (A3, b3)):
        assert Ak.data.tobytes() == A1.data.tobytes()
        np.testing.assert_array_equal(Ak.indices, A1.indices)
        np.testing.assert_array_equal(Ak.indptr, A1.indptr)
        np.testing.assert_array_equal(bk, b1)


def test_native_gzip(tmp_path):
    import gzip
    from sklearn.datasets import dump_svmlight_file
    A, b = synth.make_problem(None, seed=3, n=200, d=500, nnz=3000)
    raw = tmp_path / "r.svm"
    dump_svmlight_file(A, b, str(raw), zero_based=False)
    gz = tmp_path / "r.svm.gz"
    gz.write_bytes(gzip.compress(raw.read_bytes()))
    _same(gz)
