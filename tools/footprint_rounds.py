"""Placement spread against the hot footprint: news20-shaped
problems with a given nnz, 6 fresh handles in one process (the previous ones
kept alive, so each lands elsewhere), device Lanczos m = 100 timed per handle.  If the slow state comes from
the per-iteration footprint overflowing parts of the Infinity Cache, smaller
matrices should not show it.   python3 tools/footprint_rounds.py <nnz> ..."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for nnz in [int(v) for v in sys.argv[1:]]:
        A, b = synth.make_problem("news20", nnz=nnz)
        b01 = torch.from_numpy(np.where(b > 0, 1.0, 0.0)).to(dev)
        V = torch.empty((100, A.shape[1]), dtype=torch.float64, device=dev)
        res, keep = [], []
        for r in range(6):
            X = krcn.DeviceCSR(A, device=dev)
            x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
            Ax = X.matvec(x)
            w, g = X.weights(Ax), X.gradient(Ax, b01)
            for _ in range(2):
                X.lanczos(w, g, 100, V=V)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(8):
                X.lanczos(w, g, 100, V=V)
            torch.cuda.synchronize()
            res.append(1e6 * (time.perf_counter() - t0) / 800)
            keep.append(X)
        per = np.array(res) / (nnz / 9.1e6)
        print(f"nnz {nnz}: us/HVP {' '.join(f'{v:.1f}' for v in res)}  (per 9.1M nnz: "
              f"{' '.join(f'{v:.1f}' for v in per)})", flush=True)


if __name__ == "__main__":
    main()
