"""Per-pass format sweep on the skewed shapes: for each
(pass-1, pass-2) format pair the automatic policy could take, the HVP time
and a Lanczos step (m HVPs) on one handle.  Prints one line per pair.
    python tools/skew_formats.py [--config rcv1] [--skew] [--m 20]"""
import argparse
import re
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import synth  # noqa: E402

NAMES = {0: "auto", 1: "wave", 2: "sorted", 3: "window", 4: "jag"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="rcv1")
    ap.add_argument("--skew", action="store_true")
    ap.add_argument("--m", type=int, default=20)
    ap.add_argument("--p1", default="0,1,2,3,4")
    ap.add_argument("--p2", default="0,2,4")
    ap.add_argument("--lanes", default="0", help="pass-1 lane policies to sweep (0 auto, 1 sequential, 2..64)")
    args = ap.parse_args()
    A, b = synth.make_problem(args.config, skew=args.skew)
    dev = torch.device("cuda", 0)
    rows = np.diff(A.indptr)
    cols = np.bincount(A.indices, minlength=A.shape[1])
    print(f"{args.config}{' skew' if args.skew else ''}: {A.shape} nnz {A.nnz}; rows max {rows.max()} "
          f"mean {rows.mean():.1f}; cols max {cols.max()} mean {cols.mean():.1f}", flush=True)
    b01 = torch.from_numpy(np.where(b > 0, 1.0, 0.0)).to(dev)
    sp = lambda v: [int(x) for x in re.split(r"[,+/]", v)]  # noqa: E731 (tools/gpu.sh turns commas into spaces)
    for f1, f2, ln in [(a, c, e) for a in sp(args.p1) for c in sp(args.p2) for e in sp(args.lanes)]:
            try:
                X = krcn.DeviceCSR(A, device=dev, pass_formats=(f1 if f1 else -1, f2 if f2 else -1), lanes=(ln, 0))
                fmt = X.plan_format()
                x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
                Ax = X.matvec(x)
                w = X.weights(Ax)
                g = X.gradient(Ax, b01)
                v = (g / X.diff_norm(g)).contiguous()
                y = X.empty_d()
                for _ in range(5):
                    X.hvp(w, v, out=y)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(50):
                    X.hvp(w, v, out=y)
                torch.cuda.synchronize()
                hvp_us = 1e6 * (time.perf_counter() - t0) / 50
                V = torch.empty((args.m, A.shape[1]), dtype=torch.float64, device=dev)
                for _ in range(2):
                    X.lanczos(w, g, args.m, V=V)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    X.lanczos(w, g, args.m, V=V)
                torch.cuda.synchronize()
                lz_us = 1e6 * (time.perf_counter() - t0) / (5 * args.m)
                print(f"p1 {NAMES[f1]:7s} p2 {NAMES[f2]:7s} lanes {ln:2d} -> {fmt['pass1']:14s} {fmt['pass2']:14s} "
                      f"hvp {hvp_us:8.2f} us  lanczos {lz_us:8.2f} us/HVP ({1e6 / lz_us:9.0f} HVP/s)", flush=True)
                X.close()
            except krcn.KrcnError as e:
                print(f"p1 {NAMES[f1]:7s} p2 {NAMES[f2]:7s} lanes {ln:2d} -> refused: {str(e)[:90]}", flush=True)


if __name__ == "__main__":
    main()
