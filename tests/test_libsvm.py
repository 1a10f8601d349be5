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
