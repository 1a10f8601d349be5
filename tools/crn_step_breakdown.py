"""Where a Krylov-CRN step's time goes (GPU box): wraps the step's pieces with
device synchronisation and host timers.  usage: python tools/crn_step_breakdown.py [config] [steps]"""
import collections
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "krylov-cubic-regularized-newton_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from krcn import synth  # noqa: E402
from optimizer.cubic import Cubic_Krylov_LS  # noqa: E402
from optimizer.loss import LogisticRegression  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "news20"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
A, b = synth.make_problem(cfg)
m = synth.CONFIGS[cfg]["m"]
T = collections.defaultdict(float)
N = collections.defaultdict(int)


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        T[key] += time.perf_counter() - t0
        N[key] += 1
        return r
    setattr(obj, name, g)


loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
x0 = np.full(A.shape[1], 0.5)
Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, subspace_dim=m, tolerance=0, tqdm=False).run(x0=x0, it_max=2)
opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, subspace_dim=m, tolerance=0, tqdm=False,
                      save_first_iterations=steps + 1)
X = loss.device_matrix
for o, n, k in ((loss, "value", "value"), (loss, "gradient", "gradient"), (loss, "hess_operator", "hess_operator"),
                (X, "lanczos", "lanczos"), (opt, "_subproblem", "subproblem (host)"),
                (X, "basis_combine", "basis_combine"), (opt, "update_trace", "checkpoint"),
                (opt, "check_convergence", "check_convergence")):
    wrap(o, n, k)
torch.cuda.synchronize()
t0 = time.perf_counter()
opt.run(x0=x0, it_max=steps)
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) / steps * 1e3
print(f"{cfg} m={m}: {tot:.3f} ms per CRN step (with the per-piece synchronisation)")
acc = 0.0
for k in sorted(T, key=T.get, reverse=True):
    ms = T[k] / steps * 1e3
    acc += ms
    print(f"  {k:20s} {ms:8.3f} ms/step  ({N[k] / steps:.1f} calls/step)")
print(f"  {'rest (host loop)':20s} {tot - acc:8.3f} ms/step")
