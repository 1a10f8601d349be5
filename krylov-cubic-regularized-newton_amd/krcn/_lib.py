"""ctypes binding of libkrcn.so (the C ABI in include/krcn.h).

This is the only module that talks to the native library.  It refuses to run
without it: there is no CPU fallback anywhere on the product path.  torch is
imported first so that the library's NEEDED libamdhip64.so.7 / librccl.so.1
resolve to the copies torch already loaded (one HIP runtime per process).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("KRCN_LIB") or os.path.join(PKG_ROOT, "lib", "libkrcn.so")

# enum values of include/krcn.h
KRCN_OK = 0
KRCN_ERR_INVALID, KRCN_ERR_HIP, KRCN_ERR_RCCL, KRCN_ERR_UNSUPPORTED = 1, 2, 3, 4
KRCN_F64, KRCN_F32 = 0, 1
KRCN_SHARD_NONE, KRCN_SHARD_ROWS, KRCN_SHARD_COLS = 0, 1, 2
KRCN_LANES_AUTO, KRCN_LANES_SEQUENTIAL = 0, 1
KRCN_SLICING_AUTO, KRCN_SLICING_OFF = 0, 1
KRCN_FORMAT_AUTO, KRCN_FORMAT_WAVE, KRCN_FORMAT_SORTED, KRCN_FORMAT_WINDOW, KRCN_FORMAT_JAG = 0, 1, 2, 3, 4
KRCN_PLAN_WAVE, KRCN_PLAN_SORTED, KRCN_PLAN_WINDOW_SLICES, KRCN_PLAN_WINDOW_ACCUM = 1, 2, 3, 4
KRCN_SPACE_N, KRCN_SPACE_D = 0, 1

_STATUS_NAMES = {1: "KRCN_ERR_INVALID", 2: "KRCN_ERR_HIP", 3: "KRCN_ERR_RCCL",
                 4: "KRCN_ERR_UNSUPPORTED"}


class KrcnError(RuntimeError):
    """A libkrcn call returned a non-zero krcn_status."""

    def __init__(self, status: int, where: str, message: str):
        self.status = status
        super().__init__(f"{where}: {_STATUS_NAMES.get(status, status)}: {message}")


class CgInfo(ctypes.Structure):
    _fields_ = [("converged", ctypes.c_int), ("info", ctypes.c_int), ("iterations", ctypes.c_int),
                ("pad", ctypes.c_int), ("residual_norm", ctypes.c_double)]


class LanczosInfo(ctypes.Structure):
    _fields_ = [("m_eff", ctypes.c_int), ("breakdown", ctypes.c_int),
                ("j_break", ctypes.c_int), ("hvps", ctypes.c_int),
                ("beta_last", ctypes.c_double), ("gnorm", ctypes.c_double)]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_d = ctypes.c_double
_dp = ctypes.POINTER(ctypes.c_double)

# name -> argtypes (every symbol include/krcn.h declares)
SIGNATURES = {
    "krcn_last_error_string": [],
    "krcn_version": [],
    "krcn_csr_create": [_i, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i64, _i, ctypes.POINTER(_vp)],
    "krcn_csr_destroy": [_vp],
    "krcn_csr_owned_bytes": [_vp, ctypes.POINTER(_i64)],
    "krcn_csr_set_lanes": [_vp, _i, _i],
    "krcn_csr_set_slicing": [_vp, _i],
    "krcn_csr_set_format": [_vp, _i],
    "krcn_csr_set_pass_format": [_vp, _i, _i],
    "krcn_csr_set_graph": [_vp, _i],
    "krcn_csr_set_placement_trials": [_vp, _i],
    "krcn_csr_placement_info": [_vp, _dp],
    "krcn_csr_plan_info": [_vp, ctypes.POINTER(ctypes.c_int)],
    "krcn_csr_plan_format": [_vp, ctypes.POINTER(ctypes.c_int)],
    "krcn_csr_get_transpose": [_vp, _vp, _vp, _vp, _vp],
    "krcn_csr_attach_comm": [_vp, _vp],
    "krcn_csr_reserve": [_vp, _i, _i],
    "krcn_matvec": [_vp, _vp, _vp, _vp],
    "krcn_rmatvec": [_vp, _vp, _vp, _vp],
    "krcn_weights": [_vp, _vp, _vp, _vp],
    "krcn_hvp": [_vp, _vp, _vp, _vp, _d, _vp],
    "krcn_gradient": [_vp, _vp, _vp, _vp, _d, _vp, _vp],
    "krcn_loss_mean": [_vp, _vp, _vp, _dp, _vp],
    "krcn_loss_values": [_vp, _i, ctypes.POINTER(_vp), _vp, _dp, _vp],
    "krcn_lanczos": [_vp, _vp, _vp, _i, _i, _d, _d, _vp, _dp, _dp,
                     ctypes.POINTER(LanczosInfo), _vp],
    "krcn_basis_combine": [_vp, _i, _vp, _dp, _vp, _vp, _vp],
    "krcn_dot": [_vp, _i, _vp, _vp, _dp, _vp],
    "krcn_diff_norm": [_vp, _i, _vp, _vp, _dp, _vp],
    "krcn_comm_unique_id": [_vp],
    "krcn_comm_create": [_i, _i, _vp, _i, ctypes.POINTER(_vp)],
    "krcn_comm_destroy": [_vp],
    "krcn_comm_create_virtual": [_i, _i, ctypes.POINTER(_vp)],
    "krcn_comm_allreduce": [_vp, _i, _vp, _i64, _vp],
    "krcn_cg_solve": [_vp, _vp, _vp, _d, _d, _i, _vp, ctypes.POINTER(CgInfo), _vp],
    "krcn_vctx_create": [_i, ctypes.POINTER(_vp)],
    "krcn_vctx_destroy": [_vp],
    "krcn_lz_ext_step": [_vp, _i, _i64, _vp, _vp, _vp, _d, _vp, _dp, _vp],
    "krcn_vec_dot": [_vp, _i, _i64, _vp, _vp, _dp, _vp],
    "krcn_vec_div": [_vp, _i, _i64, _vp, _d, _vp, _vp],
    "krcn_vec_axpy": [_vp, _i, _i64, _d, _vp, _vp, _vp, _vp],
    "krcn_svm_parse": [ctypes.c_char_p, _i64, _i, ctypes.POINTER(_vp), ctypes.POINTER(_i64)],
    "krcn_svm_export": [_vp, _i64, _vp, _vp, _vp, _vp],
    "krcn_svm_destroy": [_vp],
    "krcn_prof_enable": [_vp, _i],
    "krcn_prof_read": [_vp, _dp],
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libkrcn.so once; raise ImportError (never fall back) if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libkrcn.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_char_p if name == "krcn_last_error_string" else ctypes.c_int
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    """Invoke `name` and raise KrcnError on a non-zero status."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != KRCN_OK:
        msg = lib.krcn_last_error_string()
        raise KrcnError(st, name, msg.decode() if msg else "")
