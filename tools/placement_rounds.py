"""Is the news20 slow state (DESIGN §5 placement) tied to the process or to
the allocations?  One process, 4 rounds; each round allocates a fresh
DeviceCSR (plans) and a fresh Lanczos basis V while the previous rounds'
stay alive, then times 10 device Lanczos calls (m = 100).  Also a round that
keeps the first plan but takes a fresh V, and one with a fresh plan but the
first V."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import synth  # noqa: E402


def timed(X, w, g, V, m=100, reps=10):
    for _ in range(2):
        X.lanczos(w, g, m, V=V)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        X.lanczos(w, g, m, V=V)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / (reps * m)


def main():
    A, b = synth.make_problem("news20")
    dev = torch.device("cuda", 0)
    keep = []
    b01 = torch.from_numpy(np.where(b > 0, 1.0, 0.0)).to(dev)

    def fresh_plan():
        X = krcn.DeviceCSR(A, device=dev)
        x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
        Ax = X.matvec(x)
        return X, X.weights(Ax), X.gradient(Ax, b01)

    first = None
    for r in range(4):
        X, w, g = fresh_plan()
        V = torch.empty((100, A.shape[1]), dtype=torch.float64, device=dev)
        keep.append((X, w, g, V))
        if first is None:
            first = (X, w, g, V)
        print(f"round {r}: fresh plan + fresh V: {timed(X, w, g, V):.2f} us/HVP", flush=True)
    X0, w0, g0, V0 = first
    V = torch.empty((100, A.shape[1]), dtype=torch.float64, device=dev)
    keep.append(V)
    print(f"first plan + fresh V: {timed(X0, w0, g0, V):.2f} us/HVP", flush=True)
    X, w, g = fresh_plan()
    keep.append(X)
    print(f"fresh plan + first V: {timed(X, w, g, V0):.2f} us/HVP", flush=True)
    print(f"first plan + first V: {timed(X0, w0, g0, V0):.2f} us/HVP", flush=True)
    # one plan, its scratch buffers moved one at a time (krcn_debug_realloc)
    import ctypes
    from krcn import _lib
    lib = _lib.load()
    lib.krcn_debug_realloc.argtypes = [ctypes.c_void_p, ctypes.c_int]
    names = {1: "w", 2: "u", 3: "pass-1 partials", 5: "small partials"}
    for rep in range(3):
        for which in (1, 2, 3, 5):
            assert lib.krcn_debug_realloc(X0._h, which) == 0
            print(f"first plan, fresh {names[which]}: {timed(X0, w0, g0, V0):.2f} us/HVP", flush=True)


if __name__ == "__main__":
    main()
