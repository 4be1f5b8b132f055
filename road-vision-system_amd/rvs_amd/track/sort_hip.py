"""SORT on the GPU (drop-in for src/track/sort_tracker.py).

``MultiStreamSort`` keeps the state of S independent camera streams in HBM
(per stream: a pool of tmax track slots and the list order over them) and
advances all of them by one frame per call, in place (rv_sort_update: KF
predict over every track, one workgroup per stream for the association and
bookkeeping, KF update / new tracks over every detection; f64 KF, f32 IoU,
greedy association identical to the reference's argmax loop, ground
metrics).  ``SortTracker``
is the reference's single-stream ``Tracker.update(detections, timestamp,
projector)`` on top of it, mutating and returning the same Detection objects
(sort_tracker.py:212-278).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import numpy as np
import torch

from .. import _lib
from .._lib import call, ptr, stream_ptr
from ..detect.types import Detection
from ..geometry import GroundProjector
from .base import Tracker


class MultiStreamSort:
    def __init__(self, cfg: dict, n_streams: int, tmax: int = 1024, dmax: int = 128,
                 device="cuda"):
        self.max_staleness = float(cfg.get("max_staleness", 1.0))
        self.min_hits = int(cfg.get("min_hits", 3))
        self.iou_threshold = float(cfg.get("iou_threshold", 0.3))
        self.speed_window = float(cfg.get("speed_window", 0.75))
        self.S, self.tmax, self.dmax = int(n_streams), int(tmax), int(dmax)
        self.device = torch.device(device)
        lib = _lib.load()
        nb = lib.rv_sort_state_bytes(self.S, self.tmax)
        self.state = [torch.empty(nb, dtype=torch.uint8, device=self.device)]  # updated in place
        self.cur = 0
        self.ws_bytes = lib.rv_sort_ws_bytes(self.S, self.tmax, self.dmax)
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
        self.out_id = torch.empty((self.S, self.dmax), dtype=torch.int32, device=self.device)
        self.out_dist = torch.empty((self.S, self.dmax), dtype=torch.float64, device=self.device)
        self.out_speed = torch.empty((self.S, self.dmax), dtype=torch.float64, device=self.device)
        self.params = np.zeros(6, np.float64)
        self._H = None
        self._origin = None
        self.reset()

    def reset(self):
        call("rv_sort_init", ptr(self.state[self.cur]), self.S, self.tmax, stream_ptr())

    def set_projector(self, projector: Optional[GroundProjector]):
        if projector is None:
            self._H, self._origin = None, None
            self.params[4] = -1.0
            return
        H, origin, md = projector.device_params()
        self._H = np.ascontiguousarray(H, np.float64)
        self._origin = np.ascontiguousarray(origin, np.float32)
        self.params[4] = md

    def update(self, dets: torch.Tensor, counts: torch.Tensor, ts: torch.Tensor):
        """dets (S, dmax, 6) f32, counts (S,) i32, ts (S,) f64 -- all on device.
        Returns device (track_id, distance_m, speed_kmh), each (S, dmax)."""
        self.params[:4] = [self.max_staleness, self.min_hits, self.iou_threshold,
                           self.speed_window]
        if dets.shape[1] != self.dmax:
            raise ValueError(f"dets must be (S, {self.dmax}, 6)")
        st = self.state[0]
        Hp = self._H.ctypes.data if self._H is not None else None
        op = self._origin.ctypes.data if self._origin is not None else None
        call("rv_sort_update", ptr(st), ptr(st), self.S, self.tmax, ptr(dets), ptr(counts),
             self.dmax, ptr(ts), self.params.ctypes.data, Hp, op, ptr(self.ws), self.ws_bytes,
             ptr(self.out_id), ptr(self.out_dist), ptr(self.out_speed), stream_ptr())
        return self.out_id, self.out_dist, self.out_speed

    def update_many(self, streams, timestamps) -> List[List[Detection]]:
        """Tracker.update over all S streams at once (module update_many)."""
        return update_many(self, streams, timestamps)

    def stats(self) -> dict:
        """Per-stream capacity report (rv_sort_stats), host numpy arrays:
        T (live tracks), next_id, overflow (1 once the stream had more live +
        new tracks than tmax: the tracks that did not fit were dropped and the
        stream's ids diverge from the reference's unbounded list from then
        on).  Synchronises the device."""
        T = torch.empty(self.S, dtype=torch.int32, device=self.device)
        nid = torch.empty(self.S, dtype=torch.int32, device=self.device)
        ovf = torch.empty(self.S, dtype=torch.int32, device=self.device)
        call("rv_sort_stats", ptr(self.state[self.cur]), self.S, ptr(T), ptr(nid), ptr(ovf),
             stream_ptr())
        return {"T": T.cpu().numpy(), "next_id": nid.cpu().numpy(), "overflow": ovf.cpu().numpy()}

    def check_capacity(self) -> None:
        """Raise if any stream overflowed tmax (the results are then no longer
        the reference's); call after a run, outside graph capture."""
        st = self.stats()
        bad = np.nonzero(st["overflow"])[0]
        if len(bad):
            raise _lib.RVError(f"SORT capacity: streams {bad.tolist()} exceeded tmax={self.tmax} "
                               f"live tracks (max T now {int(st['T'].max())}); construct with a "
                               "larger tmax")

    def export(self):
        """Host copy of every stream's tracks: (T[S], x[S,tmax,7], meta[S,tmax,4])."""
        x = torch.empty((self.S, self.tmax, 7), dtype=torch.float64, device=self.device)
        meta = torch.empty((self.S, self.tmax, 4), dtype=torch.int32, device=self.device)
        T = torch.empty(self.S, dtype=torch.int32, device=self.device)
        call("rv_sort_export", ptr(self.state[self.cur]), self.S, self.tmax, ptr(x), ptr(meta),
             ptr(T), stream_ptr())
        return T.cpu().numpy(), x.cpu().numpy(), meta.cpu().numpy()


def update_many(core: "MultiStreamSort", streams, timestamps) -> List[List[Detection]]:
    """Tracker.update for S camera streams in one launch: `streams` is a list
    of S detection lists (one frame per stream), `timestamps` S seconds.
    Mutates and returns the Detection objects like SortTracker.update."""
    lists = [list(x) for x in streams]
    S = core.S
    if len(lists) != S or len(timestamps) != S:
        raise ValueError(f"expected {S} streams and timestamps")
    rows = np.zeros((S, core.dmax, 6), np.float32)
    cnt = np.zeros(S, np.int32)
    for s, lst in enumerate(lists):
        if len(lst) > core.dmax:
            raise ValueError(f"{len(lst)} detections exceed dmax={core.dmax}")
        cnt[s] = len(lst)
        for i, d in enumerate(lst):
            rows[s, i] = (d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id)
    dev = core.device
    tid, dist, spd = core.update(torch.from_numpy(rows).to(dev), torch.from_numpy(cnt).to(dev),
                                 torch.tensor([float(t) for t in timestamps], dtype=torch.float64,
                                              device=dev))
    tid, dist, spd = tid.cpu().numpy(), dist.cpu().numpy(), spd.cpu().numpy()
    for s, lst in enumerate(lists):
        for i, d in enumerate(lst):
            d.track_id = None if tid[s, i] < 0 else int(tid[s, i])
            d.distance_m = None if np.isnan(dist[s, i]) else float(dist[s, i])
            d.speed_kmh = None if np.isnan(spd[s, i]) else float(spd[s, i])
    return lists


def iou_matrix_batched(trk: torch.Tensor, T: torch.Tensor, det: torch.Tensor,
                       D: torch.Tensor) -> torch.Tensor:
    """_iou_matrix (sort_tracker.py:74-80) for S streams: trk (S,Tmax,4),
    det (S,Dmax,4) f32 device, T/D (S,) int32 counts -> (S,Tmax,Dmax)."""
    S, Tmax, _ = trk.shape
    Dmax = det.shape[1]
    out = torch.empty((S, Tmax, Dmax), dtype=torch.float32, device=trk.device)
    call("rv_iou_matrix_batched", ptr(trk.contiguous()), ptr(T), ptr(det.contiguous()), ptr(D),
         ptr(out), S, Tmax, Dmax, stream_ptr())
    return out


def associate_batched(M: torch.Tensor, T: torch.Tensor, D: torch.Tensor, thr: float):
    """_associate's greedy loop (sort_tracker.py:196-208) on (S,Tmax,Dmax)
    IoU matrices (modified in place).  Returns (match_t, match_d, n_match,
    trk_match, det_match) device tensors."""
    S, Tmax, Dmax = M.shape
    mc = min(Tmax, Dmax)
    dev = M.device
    mt = torch.empty((S, mc), dtype=torch.int32, device=dev)
    md = torch.empty((S, mc), dtype=torch.int32, device=dev)
    n = torch.empty(S, dtype=torch.int32, device=dev)
    tm = torch.empty((S, Tmax), dtype=torch.int32, device=dev)
    dm = torch.empty((S, Dmax), dtype=torch.int32, device=dev)
    call("rv_greedy_assign_batched", ptr(M), ptr(T), ptr(D), S, Tmax, Dmax, float(thr), ptr(mt),
         ptr(md), ptr(n), ptr(tm), ptr(dm), stream_ptr())
    return mt, md, n, tm, dm


def project_boxes(H: torch.Tensor, boxes: torch.Tensor, origin: Optional[torch.Tensor] = None,
                  max_distance: Optional[float] = None):
    """GroundProjector.project_bbox + distance (projector.py:30-47) for n
    boxes: H (3,3) f64, boxes (n,4) f32, origin (2,) f32 -> (xy (n,2) f64,
    dist (n,) f64); NaN = None."""
    n = boxes.shape[0]
    dev = boxes.device
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    dist = torch.empty(n, dtype=torch.float64, device=dev)
    call("rv_homography_project_f64", ptr(H.contiguous()), ptr(boxes.contiguous()), n,
         ptr(origin) if origin is not None else None,
         -1.0 if max_distance is None else float(max_distance), ptr(xy), ptr(dist), stream_ptr())
    return xy, dist


class SortTracker(Tracker):
    """Single-stream reference API on the batched device tracker."""

    def __init__(self, cfg: dict, tmax: int = 1024, dmax: int = 128):
        if not torch.cuda.is_available():
            raise RuntimeError("SortTracker (HIP) needs an MI355X; there is no CPU fallback")
        self.cfg = dict(cfg)
        self.dmax = dmax
        self.tmax = tmax
        self.core = MultiStreamSort(cfg, 1, tmax=tmax, dmax=dmax)
        self._proj_key = None

    def _grow(self, n):
        # more detections than the current capacity: rebuild with room
        # (state is carried by replaying nothing -- only allowed before use)
        raise ValueError(f"{n} detections exceed dmax={self.dmax}; construct with a larger dmax")

    def update(self, detections: Iterable[Detection], timestamp: float,
               projector: Optional[GroundProjector] = None) -> List[Detection]:
        det_list = list(detections)
        for d in det_list:
            d.track_id = None
            d.distance_m = None
            d.speed_kmh = None
        if len(det_list) > self.dmax:
            self._grow(len(det_list))
        if id(projector) != self._proj_key:
            self.core.set_projector(projector)
            self._proj_key = id(projector)
        rows = np.zeros((1, self.dmax, 6), np.float32)
        for i, d in enumerate(det_list):
            rows[0, i] = (d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id)
        dev = self.core.device
        dets = torch.from_numpy(rows).to(dev)
        cnt = torch.tensor([len(det_list)], dtype=torch.int32, device=dev)
        ts = torch.tensor([float(timestamp)], dtype=torch.float64, device=dev)
        tid, dist, spd = self.core.update(dets, cnt, ts)
        tid, dist, spd = tid[0].cpu().numpy(), dist[0].cpu().numpy(), spd[0].cpu().numpy()
        for i, d in enumerate(det_list):
            d.track_id = None if tid[i] < 0 else int(tid[i])
            d.distance_m = None if np.isnan(dist[i]) else float(dist[i])
            d.speed_kmh = None if np.isnan(spd[i]) else float(spd[i])
        return det_list

    def close(self) -> None:
        self.core.reset()

