"""Repeat the 8-virtual-rank Krylov-CRN step of
tests/test_gpu_virtual_shards.py::test_synth_rows_x8_crn_step to look for the
round-3 stall (DESIGN.md §6 *The virtual-rank stall*).

Every repetition builds 8 LogisticRegression(shard=...) instances inside 8
rank threads (concurrently, as the test does; --serial builds them first in
the main thread), runs one CRN step and compute_loss_of_iterates on each, and
prints its wall time.  faulthandler dumps every thread's Python stack to
stderr when a repetition runs longer than --dump seconds, so a stall shows
where each rank was; a virtual all-reduce that times out reports the group's
state (include/krcn.h).  KRCN_LIB selects the library under test.

    python tools/virtual_stall_probe.py --reps 20 [--serial] [--dump 60]
"""
import argparse
import concurrent.futures as cf
import faulthandler
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from krcn import dist as kdist  # noqa: E402
from krcn import synth  # noqa: E402
from optimizer.cubic import Cubic_Krylov_LS  # noqa: E402
from optimizer.loss import LogisticRegression  # noqa: E402

WORLD = 8


def one_rep(A, b, serial, dev):
    mode, bounds = kdist.plan(A, WORLD, "rows")
    comms = kdist.Communicator.virtual(WORLD, dev)
    specs = [kdist.ShardSpec(A, mode, bounds, r, WORLD, comms[r]) for r in range(WORLD)]
    streams = [torch.cuda.Stream(dev) for _ in range(WORLD)]
    losses = [None] * WORLD

    def build(r):
        return LogisticRegression(A, b, l1=0, l2=0, store_mat_vec_prod=True, shard=specs[r])

    if serial:
        for r in range(WORLD):
            with torch.cuda.stream(streams[r]):
                losses[r] = build(r)

    def run(r):
        torch.cuda.set_device(dev)
        with torch.cuda.stream(streams[r]):
            loss = losses[r] if losses[r] is not None else build(r)
            opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=50, tolerance=1e-9,
                                  tqdm=False)
            tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=1)
            opt.compute_loss_of_iterates()
            out = list(tr.loss_vals)
            torch.cuda.current_stream(dev).synchronize()
            loss.device_matrix.close()
            return out

    try:
        with cf.ThreadPoolExecutor(max_workers=WORLD) as ex:
            futs = [ex.submit(run, r) for r in range(WORLD)]
            cf.wait(futs)
        res = [f.result() for f in futs]
    finally:
        for c in comms:
            c.close()
    for r in res[1:]:
        assert r == res[0], "ranks disagree"
    return res[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--dump", type=float, default=60.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    A, b = synth.make_problem("synth")
    print(f"synth problem built in {time.perf_counter() - t0:.1f} s; lib {os.environ.get('KRCN_LIB', 'in-tree')}",
          flush=True)
    for i in range(a.reps):
        faulthandler.dump_traceback_later(a.dump, repeat=True, file=sys.stderr)
        t0 = time.perf_counter()
        try:
            vals = one_rep(A, b, a.serial, dev)
            print(f"rep {i}: {time.perf_counter() - t0:.2f} s, loss values {vals}", flush=True)
        finally:
            faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
