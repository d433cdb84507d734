"""CPU-side checks of the C-ABI library (no compute calls without a GPU):
the built liblgs_hip.so loads, exports every symbol declared in include/*.h,
and reports "no device" cleanly instead of crashing."""
import ctypes as C
import glob
import os
import re

import pytest

from lgs_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="*.h"):
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", header)):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(lgs_\w+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return syms


def test_library_built():
    assert os.path.exists(abi.LIB_PATH), "run __graft_entry__.build() first"


def test_exports_every_declared_symbol():
    lib = C.CDLL(abi.LIB_PATH)
    decl = declared_symbols("lgs_hip.h")
    assert len(decl) >= 20
    missing = [s for s in sorted(decl) if not hasattr(lib, s)]
    assert not missing, f"declared but not exported: {missing}"
    # the Python binding covers every declared entry point
    assert decl == set(abi.SYMBOLS), decl.symmetric_difference(abi.SYMBOLS)


def test_host_library_exports_lgs_io_h():
    """include/lgs_io.h (f4 host components) is exported by liblgs_slam_hip.so"""
    from lgs_amd import io
    lib = io.load()
    decl = declared_symbols("lgs_io.h")
    assert len(decl) >= 7
    missing = [s for s in sorted(decl) if not hasattr(lib, s)]
    assert not missing, f"declared but not exported: {missing}"
    assert decl == set(io.SYMBOLS), decl.symmetric_difference(io.SYMBOLS)
    # every header symbol lives in one of the two libraries
    assert declared_symbols() == declared_symbols("lgs_hip.h") | decl


def test_abi_version():
    assert abi.load().lgs_abi_version() == 2


def test_no_device_is_reported_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = abi.load()
    h = C.c_void_p()
    rc = lib.lgs_ctx_create(0, C.byref(h))
    assert rc == 3 and not h.value  # LGS_ERR_NO_DEVICE


def test_null_arguments_are_rejected():
    lib = abi.load()
    assert lib.lgs_ctx_create(0, None) == 1
    assert lib.lgs_grid_precompute_max(None, None, 5, None) == 1
    assert lib.lgs_rtcsm_optimize_pose_query(None, None, None, None, None, abi.Pose2D(), None) == 1
