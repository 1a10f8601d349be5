"""Warm HVP time of one synthetic config under each storage format (auto /
forced window / ...): python tools/fmt_probe.py <config> [formats...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "krylov-cubic-regularized-newton_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "synth"
fmts = [int(f) for f in sys.argv[2:]] or [0, krcn.KRCN_FORMAT_WINDOW]
A, b = synth.make_problem(cfg)
dev = torch.device("cuda", 0)
nbytes = synth.hvp_bytes(A.shape[0], A.shape[1], A.nnz, s_val=8)
for f in fmts:
    X = krcn.DeviceCSR(A, device=dev, fmt=f)
    x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
    w = X.weights(X.matvec(x))
    v = torch.randn(A.shape[1], dtype=torch.float64, device=dev)
    y = X.empty_d()
    for _ in range(3):
        X.hvp(w, v, out=y)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for e0, e1 in evs:
        e0.record()
        X.hvp(w, v, out=y)
        e1.record()
    torch.cuda.synchronize()
    us = float(np.median([a.elapsed_time(c) * 1e3 for a, c in evs]))
    print(f"{cfg} fmt {f} {X.plan_format()} plan {X.plan_info()}: HVP {us:.1f} us = "
          f"{nbytes / us / 1e3:.0f} GB/s", flush=True)
    X.close()
