"""The C-ABI library builds, loads without a GPU, and exports exactly what
include/krcn.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "krcn.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(krcn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path():
    names = declared_functions()
    for must in ("krcn_csr_create", "krcn_hvp", "krcn_lanczos", "krcn_matvec", "krcn_gradient",
                 "krcn_weights", "krcn_loss_mean", "krcn_basis_combine", "krcn_comm_create"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from krcn import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), f"libkrcn.so does not export {name}"
    assert set(_lib.SIGNATURES) == set(declared_functions()), "ctypes signatures out of sync with krcn.h"


def test_library_is_gfx950_and_links_one_hip_runtime():
    so = os.path.join(PKG, "lib", "libkrcn.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data, "device code object for gfx950 missing"
    import subprocess
    dyn = subprocess.run(["readelf", "-d", so], capture_output=True, text=True).stdout
    assert "libamdhip64.so.7" in dyn and "librccl.so.1" in dyn
    assert "torch/lib" in dyn, "RUNPATH must point at torch's bundled ROCm runtime"


def test_calls_without_gpu_fail_cleanly():
    from krcn import _lib
    lib = _lib.load()
    assert lib.krcn_version() >= 1
    out = ctypes.c_void_p()
    # argument validation happens before any HIP call
    st = lib.krcn_csr_create(0, -1, 4, 0, None, None, None, 0, 0, 0, ctypes.byref(out))
    assert st == _lib.KRCN_ERR_INVALID
    assert b"negative" in lib.krcn_last_error_string()
    assert lib.krcn_csr_create(0, 1, 1, 0, None, None, None, 7, 0, 0, ctypes.byref(out)) == 1
    assert lib.krcn_lanczos(None, None, None, 0, 0, 0.0, 0.0, None, None, None, None, None) == 1
    with pytest.raises(_lib.KrcnError):
        _lib.call("krcn_csr_set_lanes", None, 3, 0)
