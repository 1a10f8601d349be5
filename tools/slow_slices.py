"""Which pass-1 blocks of the news20 window plan are slow, and does the set
follow the plan's memory?  (-DKRCN_WIN_TIMING build, KRCN_LIB pointing at it.)

For 3 plan instances in one process (each DeviceCSR allocated while the
previous ones stay alive, so its buffers land elsewhere), 5 matvecs each:
per block the tile-phase time (stamps 2 -> 3); prints the blocks over 1.12 x
the median in every run of an instance, as slices (block b = slice b % 128,
half b // 128), and the kernel's max / median tile time.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import _lib, synth  # noqa: E402
from win_timeline import SLOTS  # noqa: E402


def main():
    lib = _lib.load()
    lib.krcn_debug_win_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    A, b = synth.make_problem("news20")
    keep = []
    for inst in range(3):
        X = krcn.DeviceCSR(A)
        keep.append(X)
        S, _, _, grid = X.plan_info()["pass1"]
        x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=X.device)
        for _ in range(3):
            X.matvec(x)
        torch.cuda.synchronize()
        slow_sets, ratios = [], []
        for rep in range(5):
            buf = (ctypes.c_ulonglong * (3 * 2048 * SLOTS))()
            lib.krcn_debug_win_stamps(buf, 3 * 2048 * SLOTS, 1)
            X.matvec(x)
            torch.cuda.synchronize()
            lib.krcn_debug_win_stamps(buf, 3 * 2048 * SLOTS, 1)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(3, 2048, SLOTS)[0, :grid].astype(np.int64)
            t = (a[:, 3] - a[:, 2]) / 100.0
            med = np.median(t)
            slow_sets.append(set(np.nonzero(t > 1.12 * med)[0].tolist()))
            ratios.append(t.max() / med)
        always = set.intersection(*slow_sets)
        anyrun = set.union(*slow_sets)
        fmt = lambda s: " ".join(f"{bb % S}{'ab'[bb // S]}" for bb in sorted(s, key=lambda v: (v % S, v)))
        print(f"instance {inst}: max/median tile time {' '.join(f'{r:.2f}' for r in ratios)}")
        print(f"   slow in every run ({len(always)}): {fmt(always)}")
        print(f"   slow in some run ({len(anyrun)}): {fmt(anyrun)}", flush=True)


if __name__ == "__main__":
    main()
