"""Krylov-CRN run time with synchronous vs async (pinned) trace checkpoints.

usage: python tools/crn_checkpoint_ab.py [config] [it_max]   (GPU box)
Every step stores a checkpoint (save_first_iterations = it_max), so the
difference is the cost of the D2H copies in the outer loop.
"""
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
its = int(sys.argv[2]) if len(sys.argv) > 2 else 10
A, b = synth.make_problem(cfg)
m = synth.CONFIGS[cfg]["m"]


def run(async_ckpt):
    loss = LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True)
    if not async_ckpt:
        loss.to_host_async = loss.to_host
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=m, tolerance=0,
                          save_first_iterations=its + 1, tqdm=False)
    x0 = np.full(A.shape[1], 0.5)
    opt.run(x0=x0, it_max=2)   # warm: plans, workspace, pinned chunks
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=m, tolerance=0,
                          save_first_iterations=its + 1, tqdm=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr = opt.run(x0=x0, it_max=its)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / its * 1e3, np.asarray(tr.xs)


for rep in range(2):
    ms_s, xs_s = run(False)
    ms_a, xs_a = run(True)
    assert np.array_equal(xs_s, xs_a)
    print(f"{cfg} m={m}: sync checkpoints {ms_s:.2f} ms/step, async {ms_a:.2f} ms/step "
          f"({len(xs_a)} checkpoints, identical)")
