"""Which buffer's placement sets pass 1's time?  For one news20 DeviceCSR,
move one buffer at a time to a fresh allocation (debug hook) and time."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "krylov-cubic-regularized-newton_amd"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import _lib, synth  # noqa: E402

NAMES = {5: "W"}
A, b = synth.make_problem("news20")
dev = torch.device("cuda", 0)
b01 = torch.from_numpy((b > 0).astype("float64")).to(dev)
lib = _lib.load()
lib.krcn_debug_relocate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
X = krcn.DeviceCSR(A, device=dev)
x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
Ax = X.matvec(x)
w, g = X.weights(Ax), X.gradient(Ax, b01)
V = torch.empty((100, X.d), dtype=torch.float64, device=dev)
junk = []


def t1():
    X.lanczos(w, g, 100, V=V)
    X.prof_enable(True)
    for _ in range(3):
        X.lanczos(w, g, 100, V=V)
    torch.cuda.synchronize()
    p = X.prof_read()
    X.prof_enable(False)
    return 1e3 * p["pass1_kernel_ms"] / max(p["count"], 1)


print(f"base {t1():6.2f}", flush=True)
for k, name in NAMES.items():
    ts = []
    for _ in range(int(os.environ.get("RELOC_REPS", "5"))):
        junk.append(torch.empty(3 << 20, dtype=torch.uint8, device=dev))   # perturb the next allocation
        rc = lib.krcn_debug_relocate(X._h, k, 4 * (len(ts) % 2))
        if rc:
            ts.append(f"rc{rc}")
            break
        ts.append(f"{t1():6.2f}")
        print(ts[-1], flush=True)
    print(f"{name:5s} " + " ".join(ts), flush=True)
