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


def test_schedule_op_table_matches_abi():
    """rvs_amd.schedule._OPS (Python recorder) against include/rvhip.h's
    RV_SCHED_* ids and csrc/sched.hip's per-op argument counts: the recorder
    splits each call's arguments into integer / float slots exactly as the
    native issuer unpacks them."""
    from rvs_amd import _lib, schedule
    hdr = open(HEADER).read()
    ids = {m.group(2): int(m.group(1)) for m in
           re.finditer(r"#define RV_SCHED_\w+ (\d+)\s*/\* (rv_\w+) \*/", hdr)}
    src = open(os.path.join(REPO, "road-vision-system_amd", "csrc", "sched.hip")).read()
    specs = [tuple(map(int, m.groups())) for m in
             re.finditer(r"/\* RV_SCHED_\w+ \*/ \{(\d+), (\d+)\}", src)]
    assert set(ids) == set(schedule._OPS) == _lib._RECORDABLE
    for name, (op, si, host) in schedule._OPS.items():
        assert ids[name] == op, name
        argtypes = _lib._SIGS[name][1]
        assert argtypes[si] is ctypes.c_void_p, name
        nf = sum(1 for k, t in enumerate(argtypes) if k != si and t in (ctypes.c_float,
                                                                        ctypes.c_double))
        ni = len(argtypes) - 1 - nf
        assert specs[op] == (ni, nf), name
        assert all(0 <= k < len(argtypes) and k != si for k in host), name
