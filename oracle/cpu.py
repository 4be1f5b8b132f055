"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product path (road-vision-system_amd/rvs_amd) never imports it.

Each function restates one reference step; see rv_oracle.c for provenance.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or (os.path.getmtime(_SO) <
                                        os.path.getmtime(os.path.join(_HERE, "rv_oracle.c"))):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_clahe_ycrcb.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_double]
        L.oracle_clahe_u8c1.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_double]
        L.oracle_bgr2ycrcb.argtypes = [c_void_p, c_void_p, c_int]
        L.oracle_clahe_lab.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_double]
        L.oracle_bgr2lab.argtypes = [c_void_p, c_void_p, c_int]
        L.oracle_lab2bgr.argtypes = [c_void_p, c_void_p, c_int]
        L.oracle_lab_tables.argtypes = [c_void_p]
        L.oracle_nv12_to_bgr.argtypes = [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int]
        L.oracle_ycrcb2bgr.argtypes = [c_void_p, c_void_p, c_int]
        L.oracle_median_u8c3.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int]
        L.oracle_letterbox_geometry.argtypes = [c_int, c_int, c_int, c_int, POINTER(c_int)]
        L.oracle_letterbox.argtypes = [c_void_p, c_void_p, c_int, c_int, POINTER(c_int)]
        L.oracle_iou.argtypes = [c_void_p, c_void_p]
        L.oracle_iou.restype = c_float
        L.oracle_iou_matrix.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p]
        L.oracle_greedy.argtypes = [c_void_p, c_int, c_int, c_float, c_void_p, c_void_p]
        L.oracle_greedy.restype = c_int
        L.oracle_nms.argtypes = [c_void_p, c_void_p, c_int, c_double, c_int, c_void_p]
        L.oracle_nms.restype = c_int
        _lib = L
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def clahe_ycrcb(img: np.ndarray, tiles: int = 8, clip: float = 2.0) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W, _ = img.shape
    out = np.empty_like(img)
    lib().oracle_clahe_ycrcb(_p(img), _p(out), H, W, tiles, clip)
    return out


def clahe_lab(img: np.ndarray, tiles: int = 8, clip: float = 2.0) -> np.ndarray:
    """CLAHEDehaze space='LAB' (clahe_dehaze.py:21-25), see rv_oracle.c."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W, _ = img.shape
    out = np.empty_like(img)
    lib().oracle_clahe_lab(_p(img), _p(out), H, W, tiles, clip)
    return out


def bgr2lab(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_bgr2lab(_p(img), _p(out), img.size // 3)
    return out


def lab2bgr(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_lab2bgr(_p(img), _p(out), img.size // 3)
    return out


def nv12_to_bgr(y: np.ndarray, uv: np.ndarray) -> np.ndarray:
    """cv2.COLOR_YUV2BGR_NV12 (BT.601 video range, 20-bit fixed point):
    y (H, W) u8, uv (H/2, W) u8 interleaved U,V -> (H, W, 3) BGR."""
    y = np.ascontiguousarray(y, dtype=np.uint8)
    uv = np.ascontiguousarray(uv, dtype=np.uint8)
    H, W = y.shape
    out = np.empty((H, W, 3), np.uint8)
    lib().oracle_nv12_to_bgr(_p(y), _p(uv), W, W, _p(out), H, W)
    return out


LAB_TABLE_BYTES = 2 * (256 + 3072 + 512 + 4096) + 4 * 18


def lab_tables() -> bytes:
    """The oracle's 8U Lab tables, packed like rv_lab_tables_host()."""
    buf = np.zeros(LAB_TABLE_BYTES, np.uint8)
    lib().oracle_lab_tables(_p(buf))
    return buf.tobytes()


def clahe_u8c1(plane: np.ndarray, tiles: int = 8, clip: float = 2.0) -> np.ndarray:
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    out = np.empty_like(plane)
    lib().oracle_clahe_u8c1(_p(plane), _p(out), plane.shape[0], plane.shape[1], tiles, clip)
    return out


def bgr2ycrcb(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_bgr2ycrcb(_p(img), _p(out), img.size // 3)
    return out


def ycrcb2bgr(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_ycrcb2bgr(_p(img), _p(out), img.size // 3)
    return out


def median(img: np.ndarray, k: int = 3) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_median_u8c3(_p(img), _p(out), img.shape[0], img.shape[1], k)
    return out


def letterbox_geometry(H, W, imgsz=640, stride=32):
    g = (c_int * 6)()
    lib().oracle_letterbox_geometry(H, W, imgsz, stride, g)
    return tuple(int(v) for v in g)


def letterbox(img: np.ndarray, geo) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty((geo[0], geo[1], 3), np.uint8)
    lib().oracle_letterbox(_p(img), _p(out), img.shape[0], img.shape[1],
                           (c_int * 6)(*[int(v) for v in geo]))
    return out


def iou_matrix(trk: np.ndarray, det: np.ndarray) -> np.ndarray:
    trk = np.ascontiguousarray(trk, dtype=np.float32).reshape(-1, 4)
    det = np.ascontiguousarray(det, dtype=np.float32).reshape(-1, 4)
    out = np.zeros((trk.shape[0], det.shape[0]), np.float32)
    if out.size:
        lib().oracle_iou_matrix(_p(trk), trk.shape[0], _p(det), det.shape[0], _p(out))
    return out


def greedy(iou: np.ndarray, thr: float):
    m = np.array(iou, dtype=np.float32, copy=True)
    T, D = m.shape
    mt = np.zeros(max(1, min(T, D)), np.int32)
    md = np.zeros(max(1, min(T, D)), np.int32)
    n = lib().oracle_greedy(_p(m), T, D, thr, _p(mt), _p(md)) if m.size else 0
    return [(int(mt[i]), int(md[i])) for i in range(n)]


def nms(boxes: np.ndarray, scores: np.ndarray, iou_thr: float, max_keep: int) -> np.ndarray:
    boxes = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 4)
    scores = np.ascontiguousarray(scores, dtype=np.float32).reshape(-1)
    keep = np.zeros(max(1, max_keep), np.int32)
    n = lib().oracle_nms(_p(boxes), _p(scores), boxes.shape[0], float(iou_thr), max_keep,
                         _p(keep))
    return keep[:n].copy()
