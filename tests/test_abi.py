"""The C-ABI library loads and exports every symbol include/rvhip.h declares.

CPU-only: no compute call touches a GPU here (only host-side geometry and
argument validation, which return before any HIP call).
"""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "rvhip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rv_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entries():
    syms = declared_symbols()
    assert "rv_clahe_ycrcb_u8" in syms and len(syms) >= 8


def test_library_exports_every_declared_symbol():
    from rvs_amd import _lib
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"librvhip.so lacks {missing}"
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        getattr(raw, s)


def test_every_declared_symbol_has_a_python_signature():
    from rvs_amd import _lib
    import rvs_amd.kernels  # noqa: F401  (modules register their entries)
    try:
        import rvs_amd.detect.yolo_hip  # noqa: F401
        import rvs_amd.track.sort_hip  # noqa: F401
    except ImportError:
        pass
    missing = [s for s in declared_symbols() if s not in _lib._SIGS]
    assert not missing, missing


def test_abi_version_and_argument_errors():
    from rvs_amd import _lib
    lib = _lib.load()
    assert lib.rv_abi_version() >= 1
    # null pointers are rejected before any HIP call
    st = lib.rv_median_u8c3(None, None, 1, 8, 8, 24, 3, None)
    assert st == -1000
    assert b"null" in lib.rv_last_error()
    st = lib.rv_median_u8c3(1, 2, 1, 8, 8, 24, 4, None)  # even k
    assert st == -1000


@pytest.mark.parametrize("H,W", [(1080, 1920), (640, 640), (480, 640), (720, 1280), (37, 91),
                                 (2000, 300), (1, 1)])
def test_letterbox_geometry_matches_oracle(H, W):
    from rvs_amd import kernels
    from oracle import cpu
    assert kernels.letterbox_geometry(H, W) == cpu.letterbox_geometry(H, W)


def test_letterbox_geometry_known_values():
    from rvs_amd import kernels
    # 1080p -> 640x360 + 12/12 rows of 114
    assert kernels.letterbox_geometry(1080, 1920) == (384, 640, 360, 640, 12, 0)
    assert kernels.letterbox_geometry(640, 640) == (640, 640, 640, 640, 0, 0)
    assert kernels.letterbox_geometry(480, 640) == (480, 640, 480, 640, 0, 0)


def test_fused_letterbox_fits_host_only():
    """rv_clahe_median_letterbox_fits is a host query (no GPU needed)."""
    from rvs_amd import kernels
    assert kernels.clahe_median_letterbox_fits(1080, 1920, 8, 3, kernels.letterbox_geometry(1080, 1920))
    assert kernels.clahe_median_letterbox_fits(640, 640, 8, 3, kernels.letterbox_geometry(640, 640))
    assert not kernels.clahe_median_letterbox_fits(1080, 1920, 8, 5,
                                                   kernels.letterbox_geometry(1080, 1920))
