"""Two RCCL ranks: the multi-rank sharded Lanczos end to end (unique-id
broadcast, ncclCommInitRank with 2 ranks, the all-reduces inside the
recurrence) against the unsharded Lanczos of the same problem, rcv1 rows /
cols and a news20-shaped cols partition.  Rank r uses GPU min(r, visible - 1).
On a 1-GPU box both ranks land on one device, which RCCL refuses
(ncclCommInitRank -> invalid usage, "Duplicate GPU detected"): measured on
this pool, so the multi-rank path needs a 2-GPU box for this check.

python3 tools/two_ranks_one_gpu.py            (parent: starts the 2 ranks)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import numpy as np
    import torch
    import torch.distributed as tdist
    sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import krcn
    from krcn import dist as kd, synth
    rank = int(os.environ["RANK"])
    gpu = min(rank, torch.cuda.device_count() - 1)
    torch.cuda.set_device(gpu)
    tdist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)
    ok = True
    for cfg, part in (("rcv1", "cols"), ("rcv1", "rows"), ("news20", "cols")):
        A, b = synth.make_problem(cfg, n=4000 if cfg == "news20" else None, nnz=300_000 if cfg == "news20" else None)
        x = np.random.default_rng(1).uniform(-0.2, 0.2, A.shape[1])
        g = np.random.default_rng(2).standard_normal(A.shape[1])
        import scipy.special as ss
        t = A @ x
        w = ss.expit(t) * ss.expit(-t)
        X0 = krcn.DeviceCSR(A, device=dev)
        m = 30
        _, al0, be0, i0 = X0.lanczos(torch.from_numpy(w).to(dev), torch.from_numpy(g).to(dev), m)
        spec = kd.shard_problem(A, part, dev)
        X = krcn.DeviceCSR(spec.A_local, device=dev, n_global=A.shape[0], shard_mode=spec.mode)
        X.attach_comm(spec.comm)
        wl = w[spec.row_lo:spec.row_hi]
        gl = g[spec.col_lo:spec.col_hi]
        _, al, be, info = X.lanczos(torch.from_numpy(wl).to(dev), torch.from_numpy(gl).to(dev), m)
        ea = np.abs(np.asarray(al) - np.asarray(al0)).max() / np.abs(al0).max()
        eb = np.abs(np.asarray(be) - np.asarray(be0)).max() / np.abs(be0).max()
        good = ea < 1e-9 and eb < 1e-9 and info.m_eff == i0.m_eff
        ok &= good
        print(f"rank {rank} {cfg} {part}: m_eff {info.m_eff} alpha rel {ea:.2e} beta rel {eb:.2e} {'ok' if good else 'MISMATCH'}",
              flush=True)
        X.close()
        spec.comm.close()
    tdist.barrier()
    tdist.destroy_process_group()
    sys.exit(0 if ok else 1)


def parent():
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    procs = [subprocess.Popen([sys.executable, __file__, "--child"], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(2)]
    rcs = [p.wait() for p in procs]
    print("ranks exited", rcs)
    sys.exit(max(rcs))


if __name__ == "__main__":
    child() if "--child" in sys.argv else parent()
