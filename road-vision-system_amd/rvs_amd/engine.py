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

from typing import Dict, List, Optional

import numpy as np
import torch

from .config import load_config
from .detect.types import Detection
from .detect.weights import COCO80, load_weights, synthetic_weights, variant_of
from .detect.yolo_hip import YoloEngine
from .geometry import GroundProjector, build_projector
from .preprocess import PreprocessPipeline
from .track.sort_hip import MultiStreamSort


class RoadVisionEngine:
    def __init__(self, cfg: Optional[dict], n_streams: int, frame_hw, device="cuda",
                 tmax: int = 1024, projector: Optional[GroundProjector] = None,
                 weights: Optional[np.ndarray] = None):
        cfg = cfg if cfg is not None else load_config()
        self.cfg = cfg
        self.S = int(n_streams)
        self.H, self.W = int(frame_hw[0]), int(frame_hw[1])
        self.device = torch.device(device)
        self.pipeline = PreprocessPipeline(cfg.get("preprocess", {}) or {})
        det_cfg = cfg.get("detect", {}) or {}
        self.variant = variant_of(det_cfg.get("model", "yolov8n.pt"))
        if weights is None:
            wpath = det_cfg.get("weights")
            weights = load_weights(wpath, self.variant) if wpath else \
                synthetic_weights(self.variant, seed=int(det_cfg.get("seed", 0)))
        self.detector = YoloEngine(
            self.variant, weights, self.S, (self.H, self.W), imgsz=int(det_cfg.get("imgsz", 640)),
            conf=float(det_cfg.get("conf_thres", 0.25)), iou=float(det_cfg.get("iou_thres", 0.7)),
            max_det=int(det_cfg.get("max_det", 100)),
            classes_keep=[int(x) for x in det_cfg.get("classes_keep", [])], device=self.device)
        trk_cfg = cfg.get("tracking", {}) or {}
        self.tracker = MultiStreamSort(trk_cfg, self.S, tmax=tmax, dmax=self.detector.max_det,
                                       device=self.device)
        if projector is None:
            geom = cfg.get("geometry", {}) or {}
            if geom.get("enabled", False):
                projector = build_projector(geom)
        self.projector = projector
        self.tracker.set_projector(projector)
        self.proc = torch.empty((self.S, self.H, self.W, 3), dtype=torch.uint8, device=self.device)
        self.names = COCO80
        # default chain: CLAHE + median + the detector's LetterBox in one pass
        self.fused_letterbox = self.pipeline.letterbox_fusable(self.H, self.W, self.detector.geo)

    def step(self, frames: torch.Tensor, ts: torch.Tensor) -> Dict[str, torch.Tensor]:
        """frames (S,H,W,3) u8 on device, ts (S,) f64 on device."""
        if self.fused_letterbox:
            proc, lb = self.pipeline.run_with_letterbox(frames, self.detector.geo,
                                                        self.detector.lb[:frames.shape[0]])
            dets, det_n = self.detector.run_letterboxed(lb)
        else:
            proc = self.pipeline(frames)
            dets, det_n = self.detector.run(proc)
        tid, dist, spd = self.tracker.update(dets, det_n, ts)
        return {"proc": proc, "dets": dets, "det_n": det_n, "track_id": tid,
                "distance_m": dist, "speed_kmh": spd}

    def capture(self, frames: torch.Tensor, ts: torch.Tensor):
        """Record one step on (frames, ts) -- fixed device buffers -- into a
        HIP graph (torch.cuda.CUDAGraph over hipStreamBeginCapture).  Replaying
        it runs the whole step (~75 launches) with no host launch overhead or
        inter-kernel gaps from the host.  The SORT ping-pong state advances
        once per captured step, so graphs must be replayed in capture order
        (a ring of an even number of graphs over double-buffered frame
        inputs, as bench.py does).  Call step() once before the first capture
        (one-time kernel attribute setup happens outside capture)."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = self.step(frames, ts)
        return g, out

    def results(self, out: Dict[str, torch.Tensor]) -> List[List[Detection]]:
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

    def close(self):
        self.detector.close()
