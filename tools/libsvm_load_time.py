"""Load time of a news20-shaped LIBSVM file: the native multithreaded parser
(krcn_svm_parse) against sklearn's load_svmlight_file (the reference's loader,
cubic_newton.py:52-53), same file, same CSR / labels bit for bit.
python tools/libsvm_load_time.py [config] [threads] [dir]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "krylov-cubic-regularized-newton_amd"))
import numpy as np  # noqa: E402

from krcn import libsvm, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "news20"
threads = int(sys.argv[2]) if len(sys.argv) > 2 else min(16, len(os.sched_getaffinity(0)))
d = sys.argv[3] if len(sys.argv) > 3 else "/tmp"
path = os.path.join(d, f"{cfg}.svm")
if not os.path.exists(path):
    from sklearn.datasets import dump_svmlight_file
    A, b = synth.make_problem(cfg)
    dump_svmlight_file(A, b, path, zero_based=False)
size = os.path.getsize(path)
t0 = time.perf_counter()
A1, b1 = libsvm.load(path, threads=threads)
t1 = time.perf_counter()
A2, b2 = libsvm.load(path, parser="sklearn")
t2 = time.perf_counter()
same = (A1.shape == A2.shape and np.array_equal(A1.indptr, A2.indptr) and np.array_equal(A1.indices, A2.indices)
        and A1.data.tobytes() == A2.data.tobytes() and b1.tobytes() == b2.tobytes())
print(f"{cfg}: {size / 1e6:.1f} MB, {A1.shape[0]} x {A1.shape[1]}, {A1.nnz} nnz; "
      f"native ({threads} threads) {t1 - t0:.2f} s ({size / (t1 - t0) / 1e6:.0f} MB/s), "
      f"sklearn {t2 - t1:.2f} s ({size / (t2 - t1) / 1e6:.0f} MB/s): {(t2 - t1) / (t1 - t0):.1f}x; "
      f"bitwise equal: {same}")
