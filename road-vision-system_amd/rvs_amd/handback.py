"""Host side of the result hand-back (rv_results_handback).

The reference's per-frame path ends on the host: YOLOUltralytics.infer copies
``boxes.xyxy / conf / cls`` with ``.cpu().numpy()`` and builds ``Detection``
objects (src/detect/yolo_ultralytics.py:44-52), and SortTracker.update fills
``track_id / distance_m / speed_kmh`` on them (sort_tracker.py:234-247).  On
the device a step's outputs are packed into one record and copied to pinned
host memory by the step itself (csrc/results.hip); this module reads that
record and materialises the reference's ``List[Detection]`` per stream.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from . import _lib
from .detect.types import Detection

try:  # the C builder of the Detection lists (csrc/handback_py.c, built by the csrc Makefile)
    from . import _rvhandback
except ImportError:  # pragma: no cover - a checkout without the build: the numpy version
    _rvhandback = None

ROW = np.dtype([("x1", "<f4"), ("y1", "<f4"), ("x2", "<f4"), ("y2", "<f4"), ("conf", "<f4"),
                ("cls", "<i4"), ("track_id", "<i4"), ("pad", "<i4"), ("dist", "<f8"),
                ("speed", "<f8")])
assert ROW.itemsize == 48


def record_bytes(S: int, dmax: int) -> int:
    return int(_lib.load().rv_results_bytes(S, dmax))


def _header(S: int) -> int:
    return (S * 4 + 15) & ~15


class Record:
    """A pinned host record plus its device staging buffer."""

    def __init__(self, S: int, dmax: int, device, host: bool = True):
        self.S, self.dmax = int(S), int(dmax)
        self.nbytes = record_bytes(self.S, self.dmax)
        # pinned (the stream's D2H copy lands in it asynchronously) when the
        # engine lives on a GPU; a CPU-device engine (host-logic tests) gets pageable memory
        pin = torch.device(device).type == "cuda"
        self.host = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=pin) if host else None
        self.seq = 0  # hand-backs issued into this record (RoadVisionEngine.results checks it)

    def detections(self, names: Sequence[str], pool: "DetectionPool" = None) -> List[List[Detection]]:
        """The reference's Detection lists of this record (the caller must
        have synchronised the stream that filled it): built in C
        (_rvhandback) when available, else by to_detections.  With a `pool`,
        the objects are taken from its pre-made shells (DetectionPool)."""
        if _rvhandback is not None:
            return _rvhandback.build(self.host.numpy(), self.S, self.dmax, list(names), Detection,
                                     pool.items if pool is not None else None)
        return to_detections(*self.arrays(), names)

    def arrays(self):
        """(counts (S,), rows (S, dmax) structured) views of the host record.
        The caller must have synchronised the stream that filled it."""
        buf = self.host.numpy()
        n = buf[:4 * self.S].view(np.int32)
        rows = buf[_header(self.S):self.nbytes].view(ROW).reshape(self.S, self.dmax)
        return n, rows


class DetectionPool:
    """Pre-made Detection objects (every field None) for Record.detections:
    a consumer tops the pool up while it waits for the next hand-back, so
    the object and attribute-dict allocations are done before the record
    arrives and only the field values are set after it.  The objects handed
    out are ordinary Detection instances (equal to Detection(...) ones)."""

    def __init__(self):
        self.items: list = []

    def top_up(self, n: int) -> None:
        """Make shells until the pool holds at least n (no-op without the C
        builder)."""
        k = int(n) - len(self.items)
        if k > 0 and _rvhandback is not None:
            self.items.extend(_rvhandback.shells(Detection, k))


def handback(dets: torch.Tensor, det_n: torch.Tensor, track_id, distance_m, speed_kmh,
             stage: torch.Tensor, host: torch.Tensor = None) -> None:
    """Pack one step's device outputs into `stage` and (if `host` is given)
    copy them to the pinned host record, stream-ordered on the current
    stream (capturable into a HIP graph)."""
    S, dmax = dets.shape[0], dets.shape[1]
    _lib.call("rv_results_handback", _lib.ptr(dets), _lib.ptr(det_n), _lib.ptr(track_id),
              _lib.ptr(distance_m), _lib.ptr(speed_kmh), S, dmax, _lib.ptr(stage),
              stage.numel(), _lib.ptr(host), _lib.stream_ptr())


def to_detections(n: np.ndarray, rows: np.ndarray, names: Sequence[str]) -> List[List[Detection]]:
    """The reference's Detection lists (yolo_ultralytics.py:48-52 fields plus
    the tracker's track_id / distance_m / speed_kmh; NaN / -1 -> None).

    Column-wise: every field of all valid rows is converted to Python
    objects in one numpy pass, then each Detection is created without its
    generated __init__ (the dataclass keeps its fields in __dict__, so the
    objects are equal to -- and behave exactly like -- Detection(...) ones);
    ~3x faster than building them row by row, so a host consumer keeps up
    with the device (bench.py's timed region builds them)."""
    S, dmax = rows.shape
    cnt = np.clip(np.asarray(n[:S], np.int64), 0, dmax)
    r = rows[np.arange(dmax)[None, :] < cnt[:, None]]
    nn = len(names)
    kl = r["cls"].tolist()
    cname = [str(names[k]) if 0 <= k < nn else str(k) for k in kl]
    t = r["track_id"]
    tid = np.where(t < 0, None, t.astype(object)).tolist()
    d = r["dist"]
    dist = np.where(np.isnan(d), None, d.astype(object)).tolist()
    sp = r["speed"]
    spd = np.where(np.isnan(sp), None, sp.astype(object)).tolist()
    new = object.__new__
    flat = []
    app = flat.append
    for x1, y1, x2, y2, c, k, nm, ti, di, si in zip(r["x1"].tolist(), r["y1"].tolist(),
                                                    r["x2"].tolist(), r["y2"].tolist(),
                                                    r["conf"].tolist(), kl, cname, tid, dist, spd):
        o = new(Detection)
        o.__dict__ = {"x1": x1, "y1": y1, "x2": x2, "y2": y2, "conf": c, "cls_id": k,
                      "cls_name": nm, "track_id": ti, "distance_m": di, "speed_kmh": si}
        app(o)
    out = []
    i = 0
    for c in cnt.tolist():
        out.append(flat[i:i + c])
        i += c
    return out
