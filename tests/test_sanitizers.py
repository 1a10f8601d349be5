"""Host sanitizer runs of the library's multithreaded host code (SURVEY.md §5,
"Race detection"; the GPU side has no sanitizer on this pool).

`make asan` / `make tsan` (krylov-cubic-regularized-newton_amd/csrc/Makefile)
build, with g++ and AddressSanitizer + UBSan or ThreadSanitizer:
  * rendezvous_{asan,tsan}: the virtual communicator's rendezvous
    (csrc/krcn_rendezvous.hpp, the code krcn_comm_create_virtual runs) driven
    by 2, 3, 8 and 16 threads through thousands of all-reduces with a host
    sum, plus its two failure paths (a rank that never arrives, a rank that
    passes another count);
  * svm_cli_{asan,tsan}: the multithreaded svmlight parser (csrc/
    krcn_svmlight.hip) behind a command line; the inputs of
    tests/test_libsvm.py go through it and must equal sklearn's parse.
A sanitizer finding aborts the program (-fno-sanitize-recover), so every
check here is also "no report".
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "krylov-cubic-regularized-newton_amd", "csrc")
NATIVE = os.path.join(REPO, "krylov-cubic-regularized-newton_amd", "lib", "native")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")


@pytest.fixture(scope="module", autouse=True)
def built():
    r = subprocess.run(["make", "-C", CSRC, "asan", "tsan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_rendezvous_stress(san):
    r = subprocess.run([os.path.join(NATIVE, f"rendezvous_{san}"), "1500"], capture_output=True, text=True,
                       env=ENV, timeout=300)
    assert r.returncode == 0 and "rendezvous stress ok" in r.stdout, r.stdout + r.stderr[-4000:]
    assert "WARNING" not in r.stderr and "ERROR" not in r.stderr, r.stderr[-4000:]


def _cli(san, path, threads, tmp_path):
    out = tmp_path / f"out_{san}_{threads}.bin"
    r = subprocess.run([os.path.join(NATIVE, f"svm_cli_{san}"), str(path), str(threads), str(out)],
                       capture_output=True, text=True, env=ENV, timeout=300)
    assert "WARNING" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    if r.returncode == 2:
        return r.stderr.strip()
    assert r.returncode == 0, r.stderr[-4000:]
    raw = out.read_bytes()
    rows, nnz, _, _ = np.frombuffer(raw[:32], dtype=np.int64)
    o = 32
    indptr = np.frombuffer(raw[o:o + 8 * (rows + 1)], dtype=np.int64); o += 8 * (rows + 1)
    indices = np.frombuffer(raw[o:o + 8 * nnz], dtype=np.int64); o += 8 * nnz
    data = np.frombuffer(raw[o:o + 8 * nnz], dtype=np.float64); o += 8 * nnz
    labels = np.frombuffer(raw[o:o + 8 * rows], dtype=np.float64)
    return indptr, indices, data, labels


def _same_as_sklearn(san, path, threads, tmp_path):
    from sklearn.datasets import load_svmlight_file
    indptr, indices, data, labels = _cli(san, path, threads, tmp_path)
    A, b = load_svmlight_file(str(path), zero_based=True)   # unshifted, as the parser reports them
    np.testing.assert_array_equal(indptr, A.indptr)
    np.testing.assert_array_equal(indices, A.indices)
    assert data.tobytes() == A.data.tobytes()
    assert labels.tobytes() == np.asarray(b, dtype=np.float64).tobytes()


GRAMMAR = ("# header comment\n"
           "+1 qid:7 1:0.5 3:2e0 10:-1.5E-3   # trailing comment\r\n"
           "\n"
           "   -1\t2:.25 4:+7. 5:1e-320\n"
           "0.5\n"
           "-1 1:inf 2:-Infinity 3:nan 6:123456789.123456789123\n"
           "  # only a comment\n"
           "2 7:1e308 8:1e400 9:-1e-400")


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_svm_grammar(san, tmp_path):
    p = tmp_path / "g.svm"
    p.write_bytes(GRAMMAR.encode())
    _same_as_sklearn(san, p, 1, tmp_path)


@pytest.mark.parametrize("san", ["asan", "tsan"])
@pytest.mark.parametrize("line,msg", [
    ("1 3:1 2:1", "sorted and unique"),
    ("1 2:1 2:1", "sorted and unique"),
    ("1 -2:1", "Invalid index"),
    ("1 2:abc", "could not convert"),
    ("abc 2:1", "could not convert"),
    ("1 x:1", "invalid literal"),
])
def test_svm_errors(san, line, msg, tmp_path):
    p = tmp_path / "bad.svm"
    p.write_text("1 1:1\n" + line + "\n")
    err = _cli(san, p, 1, tmp_path)
    assert isinstance(err, str) and msg in err


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_svm_multithreaded_large_file(san, tmp_path):
    """A 2+ MB file cut into byte ranges for 1, 8 and 13 threads: sklearn's
    arrays every time, and no sanitizer report from the threaded parse or the
    threaded stitch."""
    from sklearn.datasets import dump_svmlight_file
    from krcn import synth
    A, b = synth.make_problem(None, seed=11, n=4000, d=50_000, nnz=300_000)
    path = tmp_path / "big.svm"
    dump_svmlight_file(A, b, str(path), zero_based=False)
    assert path.stat().st_size > (2 << 20)
    for t in (1, 8, 13):
        _same_as_sklearn(san, path, t, tmp_path)
