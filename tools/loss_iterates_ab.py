"""compute_loss_of_iterates on news20 with 100 stored iterates: the batched
device path (krcn_loss_values over the kept device copies) against the
per-iterate loop (upload + X x + loss reduction + sync per iterate), same
values bitwise.  python tools/loss_iterates_ab.py [config] [k]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "krylov-cubic-regularized-newton_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from krcn import synth  # noqa: E402
from optimizer.loss import LogisticRegression  # noqa: E402
from optimizer.opt_trace import Trace  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "news20"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
A, b = synth.make_problem(cfg)
loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
d = A.shape[1]
g = torch.Generator(device="cpu").manual_seed(0)
base = torch.full((d,), 0.5, dtype=torch.float64, device=loss.device)
tr = Trace(loss)
for i in range(k):   # iterates stored the way Optimizer.update_trace stores them
    x = base + 1e-3 * i * torch.randn(d, generator=g, dtype=torch.float64).to(loss.device)
    tr.xs.append(loss.to_host_async(x))
    tr.keep_device(tr.xs[-1], loss.keep_device_iterate(x))
loss.sync()
res = {}
for mode in ("per-iterate", "batched", "per-iterate", "batched"):
    tr.loss_vals = []
    keep = tr._dev
    if mode == "per-iterate":
        tr._dev = {}
    loss.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.compute_loss_of_iterates()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tr._dev = keep
    res.setdefault(mode, []).append((dt, np.array(tr.loss_vals)))
    print(f"{mode:12s} {k} iterates: {1e3 * dt:8.2f} ms")
assert np.array_equal(res["batched"][-1][1], res["per-iterate"][-1][1]), "values differ"
tp, tb = min(r[0] for r in res["per-iterate"]), min(r[0] for r in res["batched"])
print(f"{cfg}: per-iterate {1e3 * tp:.2f} ms, batched {1e3 * tb:.2f} ms: {tp / tb:.1f}x, values bitwise equal")
