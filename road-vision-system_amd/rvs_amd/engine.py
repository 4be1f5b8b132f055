"""Batched per-frame hot path: S camera streams x 1 frame per step.

Reproduces the reference's per-frame call order (main_preview.py:94-109):
    proc = pipeline(raw)                 -> fused CLAHE + median (HIP), which
                                            also emits the detector's letterbox
    dets = detector.infer(proc)          -> YOLOv8 + NMS (HIP)
    dets = tracker.update(dets, ts, projector)   -> SORT + geometry (HIP)
for a stream-major batch, entirely on the device: no host round trip inside a
step.  ``results()`` converts one step's device outputs into the reference's
``Detection`` lists (the only device->host copy, ~S*max_det*6 floats).
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib
from .config import load_config
from .detect.types import Detection
from .detect.weights import COCO80, variant_of, weights_from_config
from .detect.yolo_hip import YoloEngine
from .geometry import GroundProjector, build_projector
from .handback import Record, handback
from .preprocess import PreprocessPipeline
from .track.sort_hip import MultiStreamSort


class RoadVisionEngine:
    def __init__(self, cfg: Optional[dict], n_streams: int, frame_hw, device="cuda",
                 tmax: int = 1024, projector: Optional[GroundProjector] = None,
                 weights: Optional[np.ndarray] = None, lanes: int = 1, pair: int = 1):
        """pair = P >= 2: the pipelined schedule (schedule.PipelinedRun)
        runs the forwards of P consecutive steps as one batch of P*S frames
        (the small P4 / P5 layers amortise their per-launch floor; measured
        B = 64: 20.5 us per frame against 25.0 at B = 32,
        tools/probe_batch.py).  Every stream still sees its frames in order
        in SORT, so results are those of sequential step() calls; a frame's
        results come out P - 1 steps later."""
        cfg = cfg if cfg is not None else load_config()
        self.cfg = cfg
        self.S = int(n_streams)
        self.pair = max(1, int(pair))
        self.H, self.W = int(frame_hw[0]), int(frame_hw[1])
        self.device = torch.device(device)
        self.pipeline = PreprocessPipeline(cfg.get("preprocess", {}) or {})
        det_cfg = cfg.get("detect", {}) or {}
        trk_cfg = cfg.get("tracking", {}) or {}
        # main_preview.py:60-70: the detector and the tracker exist only when
        # their `enabled` key is set (src/config.py defaults both to False)
        self.detect_enabled = bool(det_cfg.get("enabled", False))
        self.tracking_enabled = bool(trk_cfg.get("enabled", False))
        self.variant = variant_of(det_cfg.get("model", "yolov8n.pt"))
        self.detector = None
        if self.detect_enabled:
            if weights is None:
                weights = weights_from_config(det_cfg, self.variant)
            self.detector = YoloEngine(
                self.variant, weights, self.S * self.pair, (self.H, self.W),
                imgsz=int(det_cfg.get("imgsz", 640)),
                conf=float(det_cfg.get("conf_thres", 0.25)),
                iou=float(det_cfg.get("iou_thres", 0.7)),
                max_det=int(det_cfg.get("max_det", 100)),
                classes_keep=[int(x) for x in det_cfg.get("classes_keep", [])],
                device=self.device, lanes=lanes)
            if self.detector.lanes > 1:
                # a multi-lane engine runs pipelined stages (schedule.PipelinedRun):
                # its forwards keep the Detect heads on the stage's own stream
                # instead of two more side streams per handle sharing the 4
                # hardware queues (r04: +3 % frames/s; RV_HEAD_STREAMS overrides)
                self.detector.set_head_streams(False)
        self.max_det = self.detector.max_det if self.detector is not None else \
            int(det_cfg.get("max_det", 100))
        # main_preview.py:64-78: a tracker or projector that fails to build
        # is reported and left off (the run goes on without that feature)
        if projector is None:
            geom = cfg.get("geometry", {}) or {}
            if geom.get("enabled", False):
                try:
                    projector = build_projector(geom)
                except Exception as exc:
                    warnings.warn(f"geometry projector init failed, running without it: {exc}")
                    projector = None
        self.projector = projector
        self.tracker = None
        if self.tracking_enabled and self.detector is not None:
            try:
                tracker = MultiStreamSort(trk_cfg, self.S, tmax=tmax, dmax=self.max_det,
                                          device=self.device)
                tracker.set_projector(projector)
                self.tracker = tracker
            except Exception as exc:
                warnings.warn(f"tracker init failed, running without it: {exc}")
                self.tracker = None
        if self.tracker is None and self.detector is not None:
            # tracker off (main_preview.py:104-109): ids and speeds stay None,
            # each detection gets projector.distance_for_bbox when a projector exists
            self._untracked = _UntrackedMetrics(self.S, self.max_det, projector, self.device)
        self.proc = torch.empty((self.S, self.H, self.W, 3), dtype=torch.uint8, device=self.device)
        self.names = COCO80
        # result hand-back: device staging buffer + the pinned host record of step()
        self.record = Record(self.S, self.max_det, self.device)
        self.rec_stage = torch.empty(self.record.nbytes, dtype=torch.uint8, device=self.device)
        # default chain: CLAHE + median + the detector's LetterBox in one pass
        self.fused_letterbox = self.detector is not None and \
            self.pipeline.letterbox_fusable(self.H, self.W, self.detector.geo)

    def _need_detector(self, what: str) -> None:
        if self.detector is None:
            raise ValueError(f"{what} needs the detector (detect.enabled is false); "
                             "step() runs the preprocess-only path")

    def preprocess_stage(self, frames: torch.Tensor, lb_slot: int = 0, lb_off: int = 0):
        """pipeline(raw) + the detector's LetterBox (main_preview.py:94-99)
        for (S,H,W,3) u8 device frames -> (proc, letterboxed batch in the
        detector's letterbox slot `lb_slot`, images [lb_off, lb_off + S))."""
        B = frames.shape[0]
        if self.fused_letterbox:
            return self.pipeline.run_with_letterbox(frames, self.detector.geo,
                                                    self.detector.lb[lb_slot][lb_off:lb_off + B])
        proc = self.pipeline(frames)
        if self.detector is None:
            return proc, None
        return proc, self.detector.letterbox(proc, lb_slot, lb_off)

    def preprocess_into(self, frames: torch.Tensor, proc: torch.Tensor, lb_slot: int = 0,
                        lb_off: int = 0) -> None:
        """preprocess_stage into a caller-owned proc buffer (rvs_amd.schedule:
        a recorded schedule must not allocate per run)."""
        B = frames.shape[0]
        if self.fused_letterbox:
            self.pipeline.run_with_letterbox(frames, self.detector.geo,
                                             self.detector.lb[lb_slot][lb_off:lb_off + B], out=proc)
            return
        if _lib._recorder is not None:
            raise RuntimeError("a recorded schedule needs the fused CLAHE+median+letterbox chain "
                               "(the unfused chain allocates and copies with torch ops)")
        p, _ = self.preprocess_stage(frames, lb_slot, lb_off)
        proc.copy_(p)

    def yolo_stage(self, lb: Optional[torch.Tensor], slot: int = 0, lane: int = 0,
                   part: int = 0, batch: Optional[int] = None) -> None:
        """YOLOv8 forward + decode in forward context `lane`; NMS candidates
        land in candidate slot `slot`.  part 1 / 2: the two halves of the
        forward (YoloEngine.forward_raw); part 2 continues part 1's batch
        (`batch` images, default S * pair)."""
        self._need_detector("yolo_stage")
        self.detector.forward_raw(lb, slot=slot, lane=lane, part=part,
                                  batch=batch if batch is not None else self.S * self.pair)

    def detect_stage(self, frames: torch.Tensor, slot: int = 0) -> torch.Tensor:
        self._need_detector("detect_stage")
        proc, lb = self.preprocess_stage(frames)
        self.yolo_stage(lb, slot)
        return proc

    def autotune(self, frames: torch.Tensor, reps: int = 3, verify: bool = False) -> int:
        """Autotune the detector's conv kernels on one batch of these frames
        (YoloEngine.autotune; pair mode: the batch of P*S the pipelined
        forwards run, the frames repeated); call outside graph capture."""
        self._need_detector("autotune")
        for h in range(self.pair):
            self.preprocess_stage(frames, 0, h * self.S)
        lb = self.detector.lb[0][:self.S * self.pair]
        return self.detector.autotune(lb, reps=reps, verify=verify)

    def track_stage(self, ts: torch.Tensor, slot: int = 0,
                    record: Optional[Record] = None) -> Dict[str, torch.Tensor]:
        """NMS of candidate slot `slot` + SORT/geometry (main_preview.py:99-109),
        then the hand-back of the results into `record` (pinned host)."""
        self._need_detector("track_stage")
        dets, det_n = self.detector.nms(ts.shape[0], slot)
        tid, dist, spd = self._metrics(dets, det_n, ts)
        out = {"dets": dets, "det_n": det_n, "track_id": tid, "distance_m": dist,
               "speed_kmh": spd}
        if record is not None:
            handback(dets, det_n, tid, dist, spd, self.rec_stage, record.host)
            record.seq += 1
            out["record"] = record
            out["seq"] = record.seq
        return out

    def track_pair_stage(self, ts_list, slot: int, records) -> List[Dict[str, torch.Tensor]]:
        """Pair mode: NMS of the P*S images of candidate slot `slot` at once,
        then SORT + hand-back of each of the P steps in order (step h owns
        images [h*S, (h+1)*S))."""
        self._need_detector("track_pair_stage")
        S = self.S
        dets, det_n = self.detector.nms(S * len(ts_list), slot)
        outs = []
        for h, (ts, rec) in enumerate(zip(ts_list, records)):
            d, n = dets[h * S:(h + 1) * S], det_n[h * S:(h + 1) * S]
            tid, dist, spd = self._metrics(d, n, ts)
            handback(d, n, tid, dist, spd, self.rec_stage, rec.host)
            outs.append({"record": rec})
        return outs

    def track_handback(self, dets: torch.Tensor, det_n: torch.Tensor, ts: torch.Tensor,
                       record: Record) -> None:
        """SORT + geometry of one step's NMS output (S images), then its
        hand-back into `record` (tracker.update + the .cpu() hand-over of
        main_preview.py:99-109)."""
        self._need_detector("track_handback")
        tid, dist, spd = self._metrics(dets, det_n, ts)
        handback(dets, det_n, tid, dist, spd, self.rec_stage, record.host)

    def _metrics(self, dets: torch.Tensor, det_n: torch.Tensor, ts: torch.Tensor):
        """(track_id, distance_m, speed_kmh) of one step's NMS output:
        SortTracker.update when tracking is enabled, else the tracker-off
        branch of main_preview.py:101-109 (rv_untracked_metrics)."""
        if self.tracker is not None:
            return self.tracker.update(dets, det_n, ts)
        return self._untracked(dets, det_n)

    def step_unit(self, frames_list, ts_list, records) -> List[Dict[str, torch.Tensor]]:
        """Pair mode, sequentially on the current stream: the preprocess of
        P consecutive steps into one letterbox slot, ONE forward over their
        P*S frames, then NMS + per-step SORT + hand-back (the work of one
        pipeline unit of schedule.PipelinedRun, each launch alone)."""
        self._need_detector("step_unit")
        S = self.S
        procs = [self.preprocess_stage(f, 0, h * S)[0] for h, f in enumerate(frames_list)]
        self.yolo_stage(self.detector.lb[0][:S * len(frames_list)], 0)
        outs = self.track_pair_stage(ts_list, 0, records)
        for o, p in zip(outs, procs):
            o["proc"] = p
        return outs

    def step(self, frames: torch.Tensor, ts: torch.Tensor,
             record: Optional[Record] = None) -> Dict[str, torch.Tensor]:
        """frames (S,H,W,3) u8 on device, ts (S,) f64 on device.  The step's
        results end in `record` (pinned host; default: the engine's own
        record, which the next step() overwrites -- read results(out) before
        it, or pass a Record per step).  With detect.enabled false only the
        preprocess runs and every stream's list is empty (main_preview.py:97-99)."""
        if self.detector is None:
            proc, _ = self.preprocess_stage(frames)
            return {"proc": proc, "no_detector": True}
        proc = self.detect_stage(frames, 0)
        out = self.track_stage(ts, 0, self.record if record is None else record)
        out["proc"] = proc
        return out

    def results(self, out: Dict[str, torch.Tensor]) -> List[List[Detection]]:
        """The reference's Detection lists of one step: from its host record
        (synchronises the device first), or from the device tensors."""
        if out.get("no_detector"):
            return [[] for _ in range(self.S)]
        if "record" in out:
            if "seq" in out and out["record"].seq != out["seq"]:
                raise RuntimeError("this step's record was overwritten by a later step(): call "
                                   "results(out) before the next step(), or pass step() its own "
                                   "Record")
            torch.cuda.synchronize(self.device)
            return out["record"].detections(self.names)
        d = out["dets"].cpu().numpy()
        n = out["det_n"].cpu().numpy()
        tid = out["track_id"].cpu().numpy()
        dist = out["distance_m"].cpu().numpy()
        spd = out["speed_kmh"].cpu().numpy()
        res = []
        for s in range(d.shape[0]):
            lst = []
            for i in range(int(n[s])):
                r = d[s, i]
                k = int(r[5])
                lst.append(Detection(float(r[0]), float(r[1]), float(r[2]), float(r[3]),
                                     float(r[4]), k, str(self.names[k]) if k < len(self.names) else str(k),
                                     None if tid[s, i] < 0 else int(tid[s, i]),
                                     None if np.isnan(dist[s, i]) else float(dist[s, i]),
                                     None if np.isnan(spd[s, i]) else float(spd[s, i])))
            res.append(lst)
        return res

    def track_stats(self) -> Dict[str, np.ndarray]:
        """Per-stream SORT capacity report (MultiStreamSort.stats); empty
        arrays when tracking is off."""
        if self.tracker is None:
            z = np.zeros(self.S, np.int32)
            return {"T": z, "next_id": z.copy(), "overflow": z.copy()}
        return self.tracker.stats()

    def close(self):
        if self.detector is not None:
            self.detector.close()


class _UntrackedMetrics:
    """The tracker-off outputs of one step (main_preview.py:101-109):
    track_id None (-1), speed_kmh None (NaN), distance_m =
    projector.distance_for_bbox(bbox) (projector.py:49-51) with a projector,
    else None -- on the device (rv_untracked_metrics), so the step's
    hand-back record is built exactly as with the tracker."""

    def __init__(self, S: int, dmax: int, projector: Optional[GroundProjector], device):
        self.S, self.dmax = int(S), int(dmax)
        self.out_id = torch.empty((self.S, self.dmax), dtype=torch.int32, device=device)
        self.out_dist = torch.empty((self.S, self.dmax), dtype=torch.float64, device=device)
        self.out_speed = torch.empty((self.S, self.dmax), dtype=torch.float64, device=device)
        self._H = self._origin = None
        self._md = -1.0
        if projector is not None:
            H, origin, md = projector.device_params()
            self._H = np.ascontiguousarray(H, np.float64)
            self._origin = np.ascontiguousarray(origin, np.float32)
            self._md = float(md)

    def __call__(self, dets: torch.Tensor, det_n: torch.Tensor):
        S = dets.shape[0]
        if S != self.S or dets.shape[1] != self.dmax:
            raise ValueError(f"dets must be ({self.S}, {self.dmax}, 6)")
        _lib.call("rv_untracked_metrics", _lib.ptr(dets), _lib.ptr(det_n), S, self.dmax,
                  self._H.ctypes.data if self._H is not None else None,
                  self._origin.ctypes.data if self._origin is not None else None, self._md,
                  _lib.ptr(self.out_id), _lib.ptr(self.out_dist), _lib.ptr(self.out_speed),
                  _lib.stream_ptr())
        return self.out_id, self.out_dist, self.out_speed
