"""Functional torch-tensor front end over the C ABI (include/rvhip.h).

Every function takes device-resident uint8 BGR frames shaped (B, H, W, 3)
(or (H, W, 3)), launches on the current torch stream and returns device
tensors.  Nothing here copies to the host or synchronises.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import call, ptr, stream_ptr


def _frames(x: torch.Tensor) -> Tuple[torch.Tensor, int, int, int, int]:
    if x.dim() == 3:
        x = x.unsqueeze(0)
    if x.dim() != 4 or x.shape[-1] != 3 or x.dtype != torch.uint8:
        raise ValueError(f"expected uint8 frames (B,H,W,3), got {tuple(x.shape)} {x.dtype}")
    if not x.is_cuda:
        raise ValueError("frames must be on the GPU (HIP path has no CPU fallback)")
    B, H, W, _ = x.shape
    if not (x.stride(3) == 1 and x.stride(2) == 3 and x.stride(0) == H * x.stride(1)):
        x = x.contiguous()
    pitch = x.stride(1)
    return x, B, H, W, pitch


def _like(x: torch.Tensor, out: Optional[torch.Tensor]) -> torch.Tensor:
    """Output frames with the same (B, H, pitch) layout as the input: the ABI
    takes one pitch for both."""
    if out is None:
        return torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=x.device)
    if out.shape != x.shape or out.stride() != x.stride():
        raise ValueError("out must have the input's shape and strides")
    return out


def clahe_ws_bytes(B: int, tiles: int) -> int:
    return int(_lib.load().rv_clahe_ws_bytes(B, tiles))


def _ws(B, tiles, ws, device):
    need = clahe_ws_bytes(B, tiles)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=device)
    return ws, need


def clahe_ycrcb(frames: torch.Tensor, tiles: int = 8, clip: float = 2.0,
                out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None):
    x, B, H, W, pitch = _frames(frames)
    out = _like(x, out)
    ws, need = _ws(B, tiles, ws, x.device)
    call("rv_clahe_ycrcb_u8", ptr(x), ptr(out), B, H, W, pitch, int(tiles), float(clip),
         ptr(ws), ws.numel(), stream_ptr())
    return out if frames.dim() == 4 else out[0]


_lab_ready = set()  # devices whose Lab tables are uploaded


def clahe_lab(frames: torch.Tensor, tiles: int = 8, clip: float = 2.0,
              out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None):
    """CLAHEDehaze space='LAB' (clahe_dehaze.py:21-25) on device frames."""
    x, B, H, W, pitch = _frames(frames)
    out = _like(x, out)
    ws, need = _ws(B, tiles, ws, x.device)
    if x.device not in _lab_ready:  # one synchronous upload per device, before capture
        with torch.cuda.device(x.device):
            call("rv_lab_init")
        _lab_ready.add(x.device)
    call("rv_clahe_lab_u8", ptr(x), ptr(out), B, H, W, pitch, int(tiles), float(clip),
         ptr(ws), ws.numel(), stream_ptr())
    return out if frames.dim() == 4 else out[0]


def nv12_to_bgr(nv12: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed NV12 frames (B, 3H/2, W) u8 on device (Y rows, then interleaved
    U,V rows) -> (B, H, W, 3) BGR, cv2.COLOR_YUV2BGR_NV12 bit for bit."""
    if nv12.dim() == 2:
        return nv12_to_bgr(nv12.unsqueeze(0), None if out is None else out.unsqueeze(0))[0]
    if nv12.dim() != 3 or nv12.dtype != torch.uint8 or not nv12.is_cuda:
        raise ValueError("expected packed NV12 uint8 (B, 3H/2, W) on the GPU")
    nv12 = nv12.contiguous()
    B, R, W = nv12.shape
    if R % 3 or (2 * R // 3) % 2 or W % 2:
        raise ValueError(f"NV12 rows {R} / width {W}: need 3H/2 rows with H, W even")
    H = 2 * R // 3
    if out is None:
        out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=nv12.device)
    elif out.shape != (B, H, W, 3) or not out.is_contiguous():
        raise ValueError("out must be a contiguous (B, H, W, 3) uint8 tensor")
    fs = R * W
    call("rv_nv12_to_bgr_u8", ptr(nv12), nv12.data_ptr() + H * W, W, W, fs, fs, ptr(out), B, H, W,
         3 * W, stream_ptr())
    return out


def median(frames: torch.Tensor, k: int = 3, out: Optional[torch.Tensor] = None):
    x, B, H, W, pitch = _frames(frames)
    out = _like(x, out)
    call("rv_median_u8c3", ptr(x), ptr(out), B, H, W, pitch, int(k), stream_ptr())
    return out if frames.dim() == 4 else out[0]


def clahe_median(frames: torch.Tensor, tiles: int = 8, clip: float = 2.0, k: int = 3,
                 out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None):
    x, B, H, W, pitch = _frames(frames)
    out = _like(x, out)
    ws, need = _ws(B, tiles, ws, x.device)
    call("rv_clahe_median_u8", ptr(x), ptr(out), B, H, W, pitch, int(tiles), float(clip),
         int(k), ptr(ws), ws.numel(), stream_ptr())
    return out if frames.dim() == 4 else out[0]


def clahe_median_letterbox(frames: torch.Tensor, tiles: int, clip: float, k: int, geo,
                           out: Optional[torch.Tensor] = None,
                           lb_out: Optional[torch.Tensor] = None,
                           ws: Optional[torch.Tensor] = None):
    """Fused CLAHE + median + LetterBox: returns (proc, letterboxed)."""
    x, B, H, W, pitch = _frames(frames)
    out = _like(x, out)
    if lb_out is None:
        lb_out = torch.empty((B, geo[0], geo[1], 3), dtype=torch.uint8, device=x.device)
    ws, need = _ws(B, tiles, ws, x.device)
    call("rv_clahe_median_letterbox_u8", ptr(x), ptr(out), B, H, W, pitch, int(tiles),
         float(clip), int(k), ptr(ws), ws.numel(), ptr(lb_out), _lib.int_array(geo), stream_ptr())
    return (out if frames.dim() == 4 else out[0]), lb_out


def clahe_median_letterbox_fits(H: int, W: int, tiles: int, k: int, geo) -> bool:
    return bool(_lib.load().rv_clahe_median_letterbox_fits(H, W, int(tiles), int(k),
                                                           _lib.int_array(geo)))


def clahe_median_fits(frames: torch.Tensor, tiles: int, k: int) -> bool:
    H, W = frames.shape[-3], frames.shape[-2]
    return bool(_lib.load().rv_clahe_median_fits(H, W, int(tiles), int(k)))


def gray_span(frames: torch.Tensor) -> torch.Tensor:
    x, B, H, W, pitch = _frames(frames)
    ws = torch.empty(2 * B, dtype=torch.int32, device=x.device)
    span = torch.empty(B, dtype=torch.int32, device=x.device)
    call("rv_gray_span_u8", ptr(x), B, H, W, pitch, ptr(ws), ptr(span), stream_ptr())
    return span


def letterbox_geometry(H: int, W: int, imgsz: int = 640, stride: int = 32):
    geo = _lib.int_array([0] * 6)
    call("rv_letterbox_geometry", H, W, imgsz, stride, geo)
    return tuple(int(v) for v in geo)


def letterbox(frames: torch.Tensor, geo, out: Optional[torch.Tensor] = None):
    x, B, H, W, pitch = _frames(frames)
    oh, ow = geo[0], geo[1]
    if out is None:
        out = torch.empty((B, oh, ow, 3), dtype=torch.uint8, device=x.device)
    call("rv_letterbox_u8", ptr(x), ptr(out), B, H, W, pitch, _lib.int_array(geo), stream_ptr())
    return out
