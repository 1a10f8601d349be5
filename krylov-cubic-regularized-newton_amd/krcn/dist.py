"""Multi-GPU sharding of the design matrix (one process per GPU).

north_star: X is partitioned across the GPUs of one node and every HVP does
one RCCL all-reduce over xGMI.  Which dimension is cut decides what that
all-reduce carries:
  rows : each rank holds a contiguous, nnz-balanced block of samples; v and
         all d-vectors are replicated; y = sum_p X_p^T (w_p * X_p v) is a
         d-length all-reduce per HVP.
  cols : each rank holds a contiguous, nnz-balanced block of features; d-vectors
         (v, the Lanczos basis, x) are sharded; X v = sum_p X_p v_p is an
         n-length all-reduce per HVP and each Lanczos dot an all-reduced scalar.
  auto : all-reduce over min(n, d) -> cols when n < d (news20), rows otherwise.
The collective runs inside libkrcn (ncclAllReduce on the kernels' stream);
torch.distributed only broadcasts the 128-byte RCCL unique id and provides the
benchmark barrier / max-over-ranks.

The planning/extraction helpers are numpy-only so the CPU test-suite can check
them with the gloo backend.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as tdist

from . import _lib
from ._lib import call
from .labels import labels01

MODES = {"none": _lib.KRCN_SHARD_NONE, "rows": _lib.KRCN_SHARD_ROWS, "cols": _lib.KRCN_SHARD_COLS}


# ------------------------------------------------------------- planning
def balanced_ranges(counts, parts):
    """Cut 0..len(counts) into `parts` contiguous ranges of ~equal sum(counts).
    Returns an int64 array of parts+1 boundaries."""
    counts = np.asarray(counts, dtype=np.int64)
    total = int(counts.sum())
    csum = np.concatenate([[0], np.cumsum(counts)])
    targets = (np.arange(1, parts) * total) // parts
    cuts = np.searchsorted(csum, targets, side="left")
    bounds = np.concatenate([[0], cuts, [len(counts)]]).astype(np.int64)
    bounds = np.maximum.accumulate(bounds)
    # every rank gets at least one row / column when there are enough of them:
    # a rank with an empty block would skip the collectives its peers wait in
    # (one dominant column, e.g. a dense bias feature, would otherwise leave
    # equal cuts behind it)
    m = len(counts)
    if m >= parts:
        for k in range(1, parts):
            bounds[k] = min(max(bounds[k], bounds[k - 1] + 1), m - (parts - k))
    return bounds


def choose_partition(n, d, world, partition="auto"):
    if world == 1:
        return "none"
    if partition == "auto":
        return "cols" if n < d else "rows"
    return partition


def plan(A, world, partition="auto"):
    """(mode, boundaries): row or column boundaries balancing nnz over ranks."""
    A = sp.csr_matrix(A)
    n, d = A.shape
    mode = choose_partition(n, d, world, partition)
    if mode == "none":
        return mode, np.array([0, n if mode == "rows" else d], dtype=np.int64)
    if mode == "rows":
        bounds = balanced_ranges(np.diff(A.indptr), world)
    else:
        bounds = balanced_ranges(np.bincount(A.indices, minlength=d), world)
    if np.any(np.diff(bounds) == 0):
        # an empty rank would skip the collectives inside the recurrence
        raise ValueError(f"cannot {mode}-partition a {n} x {d} matrix over {world} ranks: "
                         "some rank would get an empty block")
    return mode, bounds


def extract(A, mode, bounds, rank):
    """The rank's block: rows [lo, hi) or columns [lo, hi) with local column ids."""
    A = sp.csr_matrix(A)
    if mode == "none":
        return A
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    if mode == "rows":
        return A[lo:hi]
    blk = A[:, lo:hi].tocsr()
    blk.sort_indices()
    return blk


# ------------------------------------------------------------ RCCL comm
class Communicator:
    """An RCCL communicator owned by libkrcn (ncclCommInitRank)."""

    def __init__(self, world, rank, device, uid: bytes):
        self.world, self.rank = world, rank
        self.device = torch.device(device)
        self._h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, 128)
        call("krcn_comm_create", world, rank, buf, self.device.index, ctypes.byref(self._h))
        self._flag = torch.zeros(1, dtype=torch.float64, device=self.device)

    @classmethod
    def virtual(cls, world, device):
        """`world` communicators of one virtual group on `device` (krcn_comm_create_virtual):
        rank r's handle takes element r and is driven by its own host thread."""
        arr = (ctypes.c_void_p * world)()
        call("krcn_comm_create_virtual", world, torch.device(device).index, arr)
        out = []
        for r in range(world):
            c = cls.__new__(cls)
            c.world, c.rank = world, r
            c.device = torch.device(device)
            c._h = ctypes.c_void_p(arr[r])
            c._flag = torch.zeros(1, dtype=torch.float64, device=c.device)
            out.append(c)
        return out

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        call("krcn_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, device):
        """Rank 0 makes the id; torch.distributed broadcasts it."""
        world, rank = tdist.get_world_size(), tdist.get_rank()
        obj = [cls.unique_id() if rank == 0 else None]
        tdist.broadcast_object_list(obj, src=0)
        return cls(world, rank, device, obj[0])

    @property
    def handle(self):
        return self._h

    def allreduce_(self, t):
        code = _lib.KRCN_F64 if t.dtype == torch.float64 else _lib.KRCN_F32
        call("krcn_comm_allreduce", self._h, code, ctypes.c_void_p(t.data_ptr()), t.numel(),
             ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        return t

    def any(self, flag) -> bool:
        self._flag.fill_(1.0 if flag else 0.0)
        self.allreduce_(self._flag)
        return bool(self._flag.item() > 0)

    def close(self):
        if self._h.value:
            _lib.load().krcn_comm_destroy(self._h)
            self._h = ctypes.c_void_p()


class ShardSpec:
    """What LogisticRegression(shard=...) needs to run one rank's block."""

    def __init__(self, A, mode, bounds, rank, world, comm):
        self.mode_name = mode
        self.mode = MODES[mode]
        self.bounds = bounds
        self.rank, self.world, self.comm = rank, world, comm
        self.A_local = extract(A, mode, bounds, rank)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        self.row_lo, self.row_hi = (lo, hi) if mode == "rows" else (0, A.shape[0])
        self.col_lo, self.col_hi = (lo, hi) if mode == "cols" else (0, A.shape[1])

    def b_local(self, b01):
        return np.asarray(b01, dtype=np.float64)[self.row_lo:self.row_hi]


def shard_problem(A, partition="auto", device=None, rehearse=0):
    """ShardSpec for this process from torch.distributed's rank / world size.

    rehearse = N > 1 in a single process: rank 0's block of the N-way
    partition, run through the sharded code path on a 1-rank RCCL
    communicator (per-rank work and collective launch cost of an N-GPU run,
    without the cross-GPU latency)."""
    world = tdist.get_world_size() if tdist.is_initialized() else 1
    rank = tdist.get_rank() if tdist.is_initialized() else 0
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    if rehearse > 1 and world == 1:
        mode, bounds = plan(A, rehearse, partition)
        comm = Communicator(1, 0, dev, Communicator.unique_id()) if mode != "none" else None
        return ShardSpec(A, mode, bounds, 0, rehearse, comm)
    mode, bounds = plan(A, world, partition)
    comm = None
    if world > 1:
        comm = Communicator.from_torch_distributed(dev)
    return ShardSpec(A, mode, bounds, rank, world, comm)


# ---------------------------------------------------------- bench helper
class ShardedProblem:
    """Benchmark-side bundle: the rank's DeviceCSR with its communicator and
    labels, plus barrier / max-over-ranks helpers."""

    def __init__(self, A, b, dtype=torch.float64, partition="auto", device=None, rehearse=0):
        from .device import DeviceCSR
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self.world = tdist.get_world_size() if tdist.is_initialized() else 1
        self.spec = shard_problem(A, partition, self.device, rehearse=rehearse)
        self.partition = self.spec.mode_name
        n = A.shape[0]
        self.X = DeviceCSR(self.spec.A_local, device=self.device, dtype=dtype, n_global=n,
                           shard_mode=self.spec.mode)
        if self.spec.comm is not None:
            self.X.attach_comm(self.spec.comm)
        b01 = np.asarray(labels01(b), dtype=np.float64)   # loss.py:189-207 mapping
        self.b_dev = torch.from_numpy(self.spec.b_local(b01)).to(self.device, dtype)

    def full_d(self, value):
        return torch.full((self.X.d,), value, dtype=self.X.dtype, device=self.device)

    def barrier(self):
        if self.world > 1:
            tdist.barrier()

    def max_over_ranks(self, seconds):
        if self.world == 1:
            return seconds
        t = torch.tensor([seconds], dtype=torch.float64, device=self.device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        self.X.close()
        if self.spec.comm is not None:
            self.spec.comm.close()


# ------------------------------------------------------ virtual ranks
class VirtualShards:
    """A `world`-rank sharded problem on ONE GPU ("P virtual shards").

    Every rank gets its block of the same partition a `world`-GPU job uses
    (`plan`), its own DeviceCSR in the shard mode with the rank-level plans
    the auto policy picks, its own stream and a communicator of one virtual
    group (krcn_comm_create_virtual).  `run(fn)` calls fn(rank) on one host
    thread per rank, concurrently, under that rank's stream, so the library's
    collectives rendezvous exactly as across GPUs; only the transport differs
    (a device sum in rank order instead of RCCL over xGMI)."""

    def __init__(self, A, b, world, partition="auto", dtype=torch.float64, device=None):
        from .device import DeviceCSR
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        A = sp.csr_matrix(A)
        self.world = world
        self.mode, self.bounds = plan(A, world, partition)
        self.comms = Communicator.virtual(world, self.device)
        self.specs = [ShardSpec(A, self.mode, self.bounds, r, world, self.comms[r]) for r in range(world)]
        self.streams = [torch.cuda.Stream(self.device) for _ in range(world)]
        b01 = np.asarray(labels01(b), dtype=np.float64)
        self.X, self.b = [], []
        for spec in self.specs:
            X = DeviceCSR(spec.A_local, device=self.device, dtype=dtype, n_global=A.shape[0],
                          shard_mode=spec.mode)
            self.X.append(X)
            self.b.append(torch.from_numpy(spec.b_local(b01)).to(self.device, dtype))
        # attaching is collective (row shards agree on their plans: krcn.h,
        # krcn_csr_attach_comm), so every rank attaches on its own thread
        import concurrent.futures as cf

        def attach(r):
            torch.cuda.set_device(self.device)
            self.X[r].attach_comm(self.specs[r].comm)

        with cf.ThreadPoolExecutor(max_workers=world) as ex:
            for f in [ex.submit(attach, r) for r in range(world)]:
                f.result()

    def run(self, fn):
        """[fn(0), ..., fn(world-1)], each on its own thread and stream; the
        first exception is re-raised after every rank has returned."""
        import concurrent.futures as cf

        def one(r):
            torch.cuda.set_device(self.device)
            with torch.cuda.stream(self.streams[r]):
                out = fn(r)
                torch.cuda.current_stream(self.device).synchronize()
                return out

        with cf.ThreadPoolExecutor(max_workers=self.world) as ex:
            futs = [ex.submit(one, r) for r in range(self.world)]
            cf.wait(futs)
        return [f.result() for f in futs]

    def close(self):
        for X in self.X:
            X.close()
        for c in self.comms:
            c.close()
