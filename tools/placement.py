"""Is pass 1's per-process time set by where its buffers land?  Builds the
news20 DeviceCSR several times in one process (fresh allocations each time),
optionally reallocating the Lanczos operands, and prints per-launch times.
usage: python tools/placement.py [instances] [--keep-operands]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "krylov-cubic-regularized-newton_amd"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import synth  # noqa: E402

n_inst = int(sys.argv[1]) if len(sys.argv) > 1 else 6
keep = "--keep-operands" in sys.argv
A, b = synth.make_problem("news20")
dev = torch.device("cuda", 0)
b01 = torch.from_numpy((b > 0).astype("float64")).to(dev)
hold = []
ops = None
for inst in range(n_inst):
    X = krcn.DeviceCSR(A, device=dev)
    if ops is None or not keep:
        x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
        Ax = X.matvec(x)
        w = X.weights(Ax)
        g = X.gradient(Ax, b01)
        V = torch.empty((100, X.d), dtype=torch.float64, device=dev)
        ops = (w, g, V)
    w, g, V = ops
    for _ in range(int(os.environ.get("PLACE_WARM", "6"))):   # past the w placement probe (calls 1..4)
        X.lanczos(w, g, 100, V=V)
    X.prof_enable(True)
    for _ in range(4):
        X.lanczos(w, g, 100, V=V)
    torch.cuda.synchronize()
    p = X.prof_read()
    X.prof_enable(False)
    c = max(p["count"], 1)
    print(f"inst {inst}: pass1 {1e3 * p['pass1_kernel_ms'] / c:6.2f}  combine {1e3 * p['combine_ms'] / c:5.2f}"
          f"  pass2 {1e3 * p['pass2_ms'] / c:6.2f} us   V {V.data_ptr():#x} w {w.data_ptr():#x}", flush=True)
    hold.append(X)   # keep it alive so the next instance gets new addresses
