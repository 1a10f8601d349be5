"""One-process-per-GPU launcher for `bench.py --gpus N` (no torchrun needed).

`python bench.py --gpus N` without a torchrun environment re-runs the same
script as N fresh child processes with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set, exactly what
`torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1` would
export.  The parent never touches the GPU (it only counts devices, which does
not initialise HIP on this image) and never exec()s: it starts the children,
waits, and exits with the worst child status.  Asking for more GPUs than are
visible fails loudly instead of reporting a smaller run.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def in_launched_rank() -> bool:
    """True inside a torchrun / launch_ranks child (WORLD_SIZE is set)."""
    return "WORLD_SIZE" in os.environ


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    import torch
    return torch.cuda.device_count()   # counts devices without initialising HIP


def launch_ranks(nprocs: int, argv, env=None, port=None, timeout=None) -> int:
    """Run `sys.executable argv...` as `nprocs` ranks; returns the worst exit code.

    A rank that fails makes the others' collectives fail or hang, so once any
    child exits non-zero the remaining ones are terminated.  With `timeout`
    (seconds), ranks still running after it (a deadlocked collective) are
    terminated, then killed, and the call returns 124 (timeout(1)'s code)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = port or free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(nprocs):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, *argv], env=e))
    worst = 0
    pending = list(procs)
    t0 = time.monotonic()
    try:
        while pending:
            if timeout is not None and time.monotonic() - t0 > timeout:
                for q in pending:
                    q.terminate()
                for q in pending:
                    try:
                        q.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        q.kill()
                return 124
            for p in list(pending):
                try:
                    rc = p.wait(timeout=0.5)
                except subprocess.TimeoutExpired:
                    continue
                pending.remove(p)
                if rc != 0:
                    worst = worst or rc
                    for q in pending:
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return worst


def require_world(requested: int) -> None:
    """In a launched rank: the world size must be what --gpus asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != requested:
        sys.exit(f"bench: --gpus {requested} but WORLD_SIZE={world}; refusing to report a "
                 f"{world}-GPU number for a {requested}-GPU request")
