"""Frame capture front end: drop-in for src/io_video/capture.py:1-24 plus the
batched async pipeline that feeds RoadVisionEngine (README module 8).

``VideoSource(source, width, height, fps_request, backend)`` keeps the
reference's constructor, ``read() -> Frame(ok, image, ts)`` and ``release()``.
``source`` is a file: YUV4MPEG2 (``.y4m``, 4:2:0), raw NV12 (``.nv12`` /
``.yuv``, ``width`` x ``height``) or raw BGR (``.bgr``/``.raw``).  Frames are read
ahead by a native reader thread into pinned host slots (rv_capture_open) and
stamped with the wall-clock time they were read (capture.py:20).  ``image``
is H x W x 3 BGR u8: NV12 is converted on the GPU (rv_nv12_to_bgr_u8,
cv2.COLOR_YUV2BGR_NV12 bit for bit), so ``read(device=True)`` can hand the
frame over without the round trip.  Camera indices (cv2.VideoCapture(0)) and
compressed bitstreams need OpenCV / a decoder, neither of which is in this
image: they raise instead of falling back.

``MultiStreamCapture(sources, device)`` is the batched pipeline: for S
sources, ``next_batch()`` queues one frame of each as an H2D copy on a copy
stream (the slot goes back to its reader once an event recorded behind the
copy has completed; polled at the next upload), converts the NV12 batch to BGR on the device, and prefetches the
next batch while the caller runs the current one (two device buffers).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _lib
from .._lib import call, ptr, stream_ptr

RV_CAP_Y4M, RV_CAP_NV12, RV_CAP_BGR = 0, 1, 2
RV_EOF = 1
_EXT = {".y4m": RV_CAP_Y4M, ".nv12": RV_CAP_NV12, ".yuv": RV_CAP_NV12, ".bgr": RV_CAP_BGR,
        ".raw": RV_CAP_BGR}


class Frame:
    """capture.py:3-8."""
    __slots__ = ("ok", "image", "ts")

    def __init__(self, ok, image, ts):
        self.ok = ok
        self.image = image
        self.ts = ts


def write_y4m(path: str, frames_bgr: Sequence[np.ndarray], fps: int = 30) -> None:
    """Encode BGR frames as a YUV4MPEG2 4:2:0 file (BT.601 video range, the
    inverse of the NV12 conversion; chroma = 2x2 mean) -- for tests and
    synthetic camera feeds."""
    H, W = frames_bgr[0].shape[:2]
    with open(path, "wb") as f:
        f.write(f"YUV4MPEG2 W{W} H{H} F{fps}:1 Ip A1:1 C420jpeg\n".encode())
        for img in frames_bgr:
            x = img.astype(np.float32)
            b, g, r = x[..., 0], x[..., 1], x[..., 2]
            y = 16 + 0.257 * r + 0.504 * g + 0.098 * b
            u = 128 - 0.148 * r - 0.291 * g + 0.439 * b
            v = 128 + 0.439 * r - 0.368 * g - 0.071 * b
            sub = lambda p: p.reshape(H // 2, 2, W // 2, 2).mean(axis=(1, 3))
            f.write(b"FRAME\n")
            for p in (y, sub(u), sub(v)):
                f.write(np.clip(np.rint(p), 0, 255).astype(np.uint8).tobytes())


class _Reader:
    """One native reader (rv_capture_open) over a file."""

    def __init__(self, path: str, fmt: int, W: int, H: int, nbuf: int, loop: bool):
        h = ctypes.c_void_p()
        call("rv_capture_open", os.fsencode(path), fmt, W, H, nbuf, 1 if loop else 0,
             ctypes.byref(h))
        self.h = h
        info = (ctypes.c_int * 6)()
        call("rv_capture_info", h, info)
        self.W, self.H, self.fmt, self.frame_bytes, self.pinned, self.nbuf = list(info)

    def next(self):
        """(host pointer, ts, index, slot) or None at end of stream."""
        p, ts = ctypes.c_void_p(), ctypes.c_double()
        idx, slot = ctypes.c_int64(), ctypes.c_int()
        st = _lib.load().rv_capture_next(self.h, ctypes.byref(p), ctypes.byref(ts),
                                         ctypes.byref(idx), ctypes.byref(slot))
        if st == RV_EOF:
            return None
        _lib.check(st, "rv_capture_next")
        return p.value, ts.value, idx.value, slot.value

    def release(self, slot: int) -> None:
        call("rv_capture_release", self.h, slot)

    def close(self) -> None:
        if self.h:
            _lib.load().rv_capture_close(self.h)
            self.h = None


def _format_of(source, fmt: Optional[str]) -> int:
    if fmt is not None:
        return {"y4m": RV_CAP_Y4M, "nv12": RV_CAP_NV12, "bgr": RV_CAP_BGR}[fmt]
    ext = os.path.splitext(str(source))[1].lower()
    if ext not in _EXT:
        raise ValueError(f"unsupported source {source!r}: expected one of {sorted(_EXT)} "
                         "(compressed video needs a decoder, absent from this build)")
    return _EXT[ext]


class VideoSource:
    """Drop-in for capture.py:10-24 over the native reader."""

    def __init__(self, source=0, width=1280, height=720, fps_request=30, backend="auto",
                 fmt: Optional[str] = None, loop: bool = False, nbuf: int = 4, device=None):
        if isinstance(source, int):
            raise NotImplementedError(
                f"camera index {source}: live capture needs cv2.VideoCapture / V4L2, which this "
                "build does not include; pass a .y4m / .nv12 / .bgr file")
        self.fps_request = fps_request
        self.backend = backend
        self.device = torch.device(device) if device is not None else None
        self._r = _Reader(str(source), _format_of(source, fmt), int(width), int(height),
                          int(nbuf), loop)
        self.width, self.height = self._r.W, self._r.H
        self._stage = None

    def _dev(self) -> torch.device:
        if self.device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("VideoSource.read converts NV12 on the GPU; no HIP device")
            self.device = torch.device("cuda:0")
        return self.device

    def read(self, device: bool = False) -> Frame:
        """capture.py:17-20: the next frame (ok False at end of stream).
        image is BGR u8 H x W x 3: numpy, or a device tensor with device=True."""
        from ..kernels import nv12_to_bgr
        got = self._r.next()
        if got is None:
            return Frame(False, None, 0.0)
        p, ts, _, slot = got
        try:
            H, W = self.height, self.width
            host = np.ctypeslib.as_array((ctypes.c_uint8 * self._r.frame_bytes).from_address(p))
            if self._r.fmt == RV_CAP_BGR:
                img = host.reshape(H, W, 3).copy()
                if device:
                    img = torch.from_numpy(img).to(self._dev())
                return Frame(True, img, ts)
            dev = self._dev()
            if self._stage is None:
                self._stage = torch.empty((3 * H // 2, W), dtype=torch.uint8, device=dev)
            self._stage.copy_(torch.from_numpy(host.reshape(3 * H // 2, W)))
            img = nv12_to_bgr(self._stage)
            return Frame(True, img if device else img.cpu().numpy(), ts)
        finally:
            self._r.release(slot)

    def release(self):
        if self._r is not None:
            self._r.close()
            self._r = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class MultiStreamCapture:
    """S file sources -> stream-major device batches (S, H, W, 3) u8 plus the
    per-stream read times, for RoadVisionEngine.step.  Uploads run on their
    own stream and one batch ahead of the caller."""

    def __init__(self, sources: Sequence[str], device="cuda", fmt: Optional[str] = None,
                 width: int = 0, height: int = 0, loop: bool = False, nbuf: int = 4,
                 prefetch: bool = True):
        self.device = torch.device(device)
        fmts = [_format_of(s, fmt) for s in sources]
        if len(set(fmts)) != 1:
            raise ValueError("all sources must have the same format")
        self.readers: List[_Reader] = [_Reader(str(s), fmts[0], width, height, nbuf, loop)
                                       for s in sources]
        r0 = self.readers[0]
        if any((r.W, r.H) != (r0.W, r0.H) for r in self.readers):
            raise ValueError("all sources must have the same frame size")
        self.S, self.H, self.W, self.fmt = len(sources), r0.H, r0.W, r0.fmt
        self.frame_bytes = r0.frame_bytes
        self.pinned = all(r.pinned for r in self.readers)
        self._handles = (ctypes.c_void_p * self.S)(*[r.h.value for r in self.readers])
        self.copy_stream = torch.cuda.Stream(self.device)
        nv = 2 if prefetch else 1
        raw_shape = (self.S, self.frame_bytes)
        self._raw = [torch.empty(raw_shape, dtype=torch.uint8, device=self.device)
                     for _ in range(nv)]
        self._bgr = [torch.empty((self.S, self.H, self.W, 3), dtype=torch.uint8,
                                 device=self.device) for _ in range(nv)]
        self._ts = [np.zeros(self.S, np.float64) for _ in range(nv)]
        self._idx = [np.zeros(self.S, np.int64) for _ in range(nv)]
        self._ready = [torch.cuda.Event() for _ in range(nv)]
        self._pending = [False] * nv
        self._k = 0
        self.prefetch = prefetch
        self.done = False
        if prefetch:
            self._pending[0] = self._issue(0)

    def _issue(self, j: int) -> bool:
        """Queue batch j's uploads + conversion on the copy stream."""
        from ..kernels import nv12_to_bgr
        with torch.cuda.stream(self.copy_stream):
            st = _lib.load().rv_capture_upload_batch(
                self._handles, self.S, ptr(self._raw[j]), self.frame_bytes,
                self._ts[j].ctypes.data, self._idx[j].ctypes.data,
                stream_ptr(self.copy_stream))
            if st == RV_EOF:
                return False
            _lib.check(st, "rv_capture_upload_batch")
            if self.fmt == RV_CAP_BGR:
                self._bgr[j].view(self.S, -1).copy_(self._raw[j])
            else:
                nv12_to_bgr(self._raw[j].view(self.S, 3 * self.H // 2, self.W), out=self._bgr[j])
            self._ready[j].record(self.copy_stream)
        return True

    def next_batch(self):
        """(frames (S,H,W,3) u8, ts (S,) f64 device tensor, frame indices
        (S,) int64 numpy) or None at the end of any stream.  The returned
        frames stay valid for the work the caller issues on the current stream
        before its next call (two buffers; the refill waits for that work)."""
        if self.done:
            return None
        nv = len(self._raw)
        j = self._k % nv
        if not self.prefetch:
            self._pending[j] = self._issue(j)
        if not self._pending[j]:
            self.done = True
            return None
        if self.prefetch:  # start the next batch's uploads before handing this one out
            # into the buffers handed out by the previous call: the copy stream
            # waits for the work the caller has issued on them so far
            consumed = torch.cuda.Event()
            consumed.record(torch.cuda.current_stream(self.device))
            self.copy_stream.wait_event(consumed)
            self._pending[(j + 1) % nv] = self._issue((j + 1) % nv)
        torch.cuda.current_stream(self.device).wait_event(self._ready[j])
        self._k += 1
        ts = torch.from_numpy(self._ts[j].copy()).to(self.device, non_blocking=False)
        return self._bgr[j], ts, self._idx[j].copy()

    def close(self):
        torch.cuda.synchronize(self.device)
        for r in self.readers:
            r.close()
        self.readers = []

    def __del__(self):
        try:
            if self.readers:
                self.close()
        except Exception:
            pass
