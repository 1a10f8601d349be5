"""Timeline of the LDS-window passes from a -DKRCN_WIN_TIMING build
(make variant V=9 EXTRA_FLAGS=-DKRCN_WIN_TIMING; run with KRCN_LIB pointing at it).

For pass 1 (X z, krcn_matvec) and pass 2 (X^T u, krcn_rmatvec) on the
news20-shaped matrix (or the config named by argv[1]): per block, entry / prologue / segment window-ready and
tiles-done / per-wave finish stamps (s_memrealtime, 10 ns), summarised as
distributions relative to the earliest block entry.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
import torch  # noqa: E402

import krcn  # noqa: E402
from krcn import _lib, synth  # noqa: E402

SLOTS = 32


def stamps(lib, grid, table):
    """table 0: slices-mode launches (pass over X), 1: accumulate mode or the single-window jagged pass (X^T)."""
    buf = (ctypes.c_ulonglong * (3 * 2048 * SLOTS))()
    assert lib.krcn_debug_win_stamps(buf, 3 * 2048 * SLOTS, 1) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(3, 2048, SLOTS)[table, :grid].astype(np.int64)
    return a


def summarize(name, a):
    # s_memrealtime runs with a fixed offset per XCD (tools/dispatch_microbench.hip:
    # waves of one XCD start within 0.24 us, XCD offsets 0-2 us and stable), so
    # stamps are taken relative to the first entry on the block's XCD (b % 8)
    ok = a[:, 0] > 0
    x0 = np.zeros(8, dtype=np.int64)
    for x in range(8):
        m = ok & (np.arange(a.shape[0]) % 8 == x)
        x0[x] = a[m, 0].min() if m.any() else 0
    a = a.copy()
    base = x0[np.arange(a.shape[0]) % 8][:, None]
    a = np.where(a > 0, a - base, 0)
    a = a[ok]
    if a.shape[0] == 0:
        print(f"== {name}: no stamps (the pass runs another format)")
        return
    rel = lambda v: v / 100.0   # us
    q = lambda v: f"p0 {np.min(v):7.2f} p50 {np.median(v):7.2f} p90 {np.percentile(v, 90):7.2f} max {np.max(v):7.2f}"
    print(f"== {name}: {a.shape[0]} blocks; us from the first block entry on the block's XCD")
    print(" entry      ", q(rel(a[:, 0])))
    print(" prologue   ", q(rel(a[:, 1])))
    for i in range(4):
        m = a[:, 2 + 2 * i] > 0
        if m.sum() == 0:
            continue
        print(f" seg{i} ready  ", q(rel(a[m, 2 + 2 * i])), f"({m.sum()} blocks)")
        print(f" seg{i} tiles  ", q(rel(a[m, 3 + 2 * i])))
        print(f" seg{i} tiles-ready", q((a[m, 3 + 2 * i] - a[m, 2 + 2 * i]) / 100.0))
    w = a[:, 16:32]
    wr = rel(w)
    spread = (w.max(1) - w.min(1)) / 100.0
    print(" wave done  ", q(wr.ravel()))
    print(" wave spread", q(spread))
    print(" end        ", q(rel(a[:, 10])))
    # per-XCD (block % 8) and per block-in-slice (b // 128 for a 128-slice plan) medians
    idx = np.nonzero(ok)[0]
    xcd = idx % 8
    print(" end by XCD    ", " ".join(f"{np.median(rel(a[xcd == x, 10])):6.2f}" for x in range(8)))
    print(" tiles by XCD  ", " ".join(f"{np.median((a[xcd == x, 3] - a[xcd == x, 2]) / 100.0):6.2f}" for x in range(8)))
    slow = idx[np.argsort(-a[:, 10])[:12]]
    print(" slowest blocks", " ".join(str(int(v)) for v in slow))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "news20"   # any krcn.synth config (rcv1: jagged pass 2 stamps)
    lib = _lib.load()
    lib.krcn_debug_win_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    A, b = synth.make_problem(cfg)
    X = krcn.DeviceCSR(A)
    print("formats", X.plan_format(), "plan", X.plan_info())
    dev = X.device
    x = torch.full((A.shape[1],), 0.5, dtype=torch.float64, device=dev)
    u = torch.randn(A.shape[0], dtype=torch.float64, device=dev)
    for _ in range(3):
        X.matvec(x)
        X.rmatvec(u)
    torch.cuda.synchronize()
    g1, g2 = X.plan_info()["pass1"][3], X.plan_info()["pass2"][3]
    stamps(lib, 1, 0)
    X.matvec(x)
    torch.cuda.synchronize()
    summarize("pass 1 (X z, slices), krcn_matvec", stamps(lib, g1, 0))
    X.rmatvec(u)
    torch.cuda.synchronize()
    summarize("pass 2 (X^T u: window-accum or single-window jagged), krcn_rmatvec", stamps(lib, g2, 1))
    # inside the Lanczos recurrence (the bench workload): the last step's launches
    Ax = X.matvec(x)
    w = X.weights(Ax)
    bvec = torch.from_numpy(np.where(b > 0, 1.0, 0.0)).to(dev)
    gr = X.gradient(Ax, bvec)
    V = torch.empty((8, A.shape[1]), dtype=torch.float64, device=dev)
    X.lanczos(w, gr, 8, V=V)
    torch.cuda.synchronize()
    stamps(lib, 1, 0)
    X.lanczos(w, gr, 8, V=V)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (3 * 2048 * SLOTS))()
    assert lib.krcn_debug_win_stamps(buf, 3 * 2048 * SLOTS, 1) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(3, 2048, SLOTS).astype(np.int64)
    summarize("pass 1 in krcn_lanczos (last launch, final quotient)", a[0, :g1])
    if a[2, :, 0].any():
        summarize("pass 1 in krcn_lanczos (fused step B, last loop step)", a[2, :g1])
    summarize("pass 2 in krcn_lanczos (last launch)", a[1, :g2])


if __name__ == "__main__":
    main()
