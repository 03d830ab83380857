"""CPU tests of the drop-in boundary: libmmt.so loads (no GPU needed) and exports every entry
point declared in include/mmt.h; the Python plumbing refuses to run without it."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mmt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmt_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_boundary():
    syms = declared_symbols()
    for s in ("mmt_create", "mmt_destroy", "mmt_orb_extract", "mmt_orb_extract_batch",
              "mmt_orb_extract_device", "mmt_last_error", "mmt_version"):
        assert s in syms


def test_library_exports_all_declared_symbols():
    import multimot_track_amd as M
    if not os.path.exists(M.LIB_PATH):
        from multimot_track_amd import build as B
        B.build()
    lib = ctypes.CDLL(M.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.mmt_version() >= 100


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import multimot_track_amd as M
    with pytest.raises(M.MmtError):
        M.Context(M.kitti03_config())


def test_every_called_entry_point_has_argtypes():
    """Every mmt_* entry point the Python plumbing calls declares its ctypes argtypes (without
    them ctypes passes the 64-bit context handle as a C int, a host segfault on the GPU box)."""
    src = open(os.path.join(ROOT, "multimot_track_amd", "__init__.py")).read()
    called = set(re.findall(r"lib\(\)\.(mmt_\w+)\(", src))
    declared = set(re.findall(r"L\.(mmt_\w+)\.argtypes", src))
    assert called and not called - declared, sorted(called - declared)
