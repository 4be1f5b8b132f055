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

import contextlib
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import load_config
from .detect.types import Detection
from .detect.weights import COCO80, variant_of, weights_from_config
from .detect.yolo_hip import YoloEngine
from .geometry import GroundProjector, build_projector
from .handback import Record, handback, to_detections
from .preprocess import PreprocessPipeline
from .track.sort_hip import MultiStreamSort


class RoadVisionEngine:
    def __init__(self, cfg: Optional[dict], n_streams: int, frame_hw, device="cuda",
                 tmax: int = 1024, projector: Optional[GroundProjector] = None,
                 weights: Optional[np.ndarray] = None, lanes: int = 1, pair: int = 1):
        """pair = P >= 2: the pipelined schedule (OverlappedSteps depth 4)
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
        self.variant = variant_of(det_cfg.get("model", "yolov8n.pt"))
        if weights is None:
            weights = weights_from_config(det_cfg, self.variant)
        self.detector = YoloEngine(
            self.variant, weights, self.S * self.pair, (self.H, self.W),
            imgsz=int(det_cfg.get("imgsz", 640)),
            conf=float(det_cfg.get("conf_thres", 0.25)), iou=float(det_cfg.get("iou_thres", 0.7)),
            max_det=int(det_cfg.get("max_det", 100)),
            classes_keep=[int(x) for x in det_cfg.get("classes_keep", [])], device=self.device,
            lanes=lanes)
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
        # result hand-back: device staging buffer + the pinned host record of step()
        self.record = Record(self.S, self.detector.max_det, self.device)
        self.rec_stage = torch.empty(self.record.nbytes, dtype=torch.uint8, device=self.device)
        # default chain: CLAHE + median + the detector's LetterBox in one pass
        self.fused_letterbox = self.pipeline.letterbox_fusable(self.H, self.W, self.detector.geo)

    def preprocess_stage(self, frames: torch.Tensor, lb_slot: int = 0, lb_off: int = 0):
        """pipeline(raw) + the detector's LetterBox (main_preview.py:94-99)
        for (S,H,W,3) u8 device frames -> (proc, letterboxed batch in the
        detector's letterbox slot `lb_slot`, images [lb_off, lb_off + S))."""
        B = frames.shape[0]
        if self.fused_letterbox:
            return self.pipeline.run_with_letterbox(frames, self.detector.geo,
                                                    self.detector.lb[lb_slot][lb_off:lb_off + B])
        proc = self.pipeline(frames)
        return proc, self.detector.letterbox(proc, lb_slot, lb_off)

    def yolo_stage(self, lb: Optional[torch.Tensor], slot: int = 0, lane: int = 0,
                   part: int = 0) -> None:
        """YOLOv8 forward + decode in forward context `lane`; NMS candidates
        land in candidate slot `slot`.  part 1 / 2: the two halves of the
        forward (YoloEngine.forward_raw)."""
        self.detector.forward_raw(lb, slot=slot, lane=lane, part=part,
                                  batch=self.S if lb is not None else self.S * self.pair)

    def detect_stage(self, frames: torch.Tensor, slot: int = 0) -> torch.Tensor:
        proc, lb = self.preprocess_stage(frames)
        self.yolo_stage(lb, slot)
        return proc

    def autotune(self, frames: torch.Tensor, reps: int = 3, verify: bool = False) -> int:
        """Autotune the detector's conv kernels on one batch of these frames
        (YoloEngine.autotune; pair mode: the batch of P*S the pipelined
        forwards run, the frames repeated); call outside graph capture."""
        for h in range(self.pair):
            self.preprocess_stage(frames, 0, h * self.S)
        lb = self.detector.lb[0][:self.S * self.pair]
        return self.detector.autotune(lb, reps=reps, verify=verify)

    def track_stage(self, ts: torch.Tensor, slot: int = 0,
                    record: Optional[Record] = None) -> Dict[str, torch.Tensor]:
        """NMS of candidate slot `slot` + SORT/geometry (main_preview.py:99-109),
        then the hand-back of the results into `record` (pinned host)."""
        dets, det_n = self.detector.nms(ts.shape[0], slot)
        tid, dist, spd = self.tracker.update(dets, det_n, ts)
        out = {"dets": dets, "det_n": det_n, "track_id": tid, "distance_m": dist,
               "speed_kmh": spd}
        if record is not None:
            handback(dets, det_n, tid, dist, spd, self.rec_stage, record.host)
            out["record"] = record
        return out

    def track_pair_stage(self, ts_list, slot: int, records) -> List[Dict[str, torch.Tensor]]:
        """Pair mode: NMS of the P*S images of candidate slot `slot` at once,
        then SORT + hand-back of each of the P steps in order (step h owns
        images [h*S, (h+1)*S))."""
        S = self.S
        dets, det_n = self.detector.nms(S * len(ts_list), slot)
        outs = []
        for h, (ts, rec) in enumerate(zip(ts_list, records)):
            d, n = dets[h * S:(h + 1) * S], det_n[h * S:(h + 1) * S]
            tid, dist, spd = self.tracker.update(d, n, ts)
            handback(d, n, tid, dist, spd, self.rec_stage, rec.host)
            outs.append({"record": rec})
        return outs

    def step_unit(self, frames_list, ts_list, records) -> List[Dict[str, torch.Tensor]]:
        """Pair mode, sequentially on the current stream: the preprocess of
        P consecutive steps into one letterbox slot, ONE forward over their
        P*S frames, then NMS + per-step SORT + hand-back (the work of one
        pipeline unit of OverlappedSteps, each launch alone)."""
        S = self.S
        procs = [self.preprocess_stage(f, 0, h * S)[0] for h, f in enumerate(frames_list)]
        self.yolo_stage(self.detector.lb[0][:S * len(frames_list)], 0)
        outs = self.track_pair_stage(ts_list, 0, records)
        for o, p in zip(outs, procs):
            o["proc"] = p
        return outs

    def step(self, frames: torch.Tensor, ts: torch.Tensor) -> Dict[str, torch.Tensor]:
        """frames (S,H,W,3) u8 on device, ts (S,) f64 on device.  The step's
        results end in self.record (pinned host), read by results()."""
        proc = self.detect_stage(frames, 0)
        out = self.track_stage(ts, 0, self.record)
        out["proc"] = proc
        return out

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
        """The reference's Detection lists of one step: from its host record
        (synchronises the device first), or from the device tensors."""
        if "record" in out:
            torch.cuda.synchronize(self.device)
            n, rows = out["record"].arrays()
            return to_detections(n, rows, self.names)
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
        """Per-stream SORT capacity report (MultiStreamSort.stats)."""
        return self.tracker.stats()

    def close(self):
        self.detector.close()



class OverlappedSteps:
    """K captured steps whose stages overlap across steps.

    A step is three stages with different bottlenecks: preprocess P (CLAHE +
    median + letterbox: VALU-bound streaming), yolo Y (the conv stack:
    LDS/MFMA/latency-bound) and track T (NMS + SORT: one workgroup per frame /
    camera stream, latency-bound and nearly idle on 256 CUs).  Consecutive
    steps only share state through T (SORT is sequential per stream), so with
    `depth=3` graph j runs  Y(j) || P(j+1) || T(j-1)  on three streams (the
    letterbox batch and the NMS candidates are double-buffered by step
    parity); with `depth=2` it runs  [T(j-1) || P(j)] -> Y(j).  A prologue /
    epilogue graph fills and drains the pipeline.  Replayed in order, the K
    steps give the same results as K step() calls (tests/test_engine_gpu.py).

    With an engine of pair = P > 1 (depth 4 only) a pipeline unit is P
    consecutive steps: one forward over their P*S frames, then NMS and the P
    steps' SORT + hand-back in step order (`chunk` counts units; the default
    keeps 8 steps per graph).

    Each step's T stage ends with the result hand-back into that step's own
    pinned host record (outs[k]["record"]), so every outs[k] holds step k's
    detections and track ids after run(); outs[k]["proc"] is step k's proc
    batch.  The device tensors of the NMS / SORT outputs are shared by all
    steps and are not kept in outs."""

    def __init__(self, eng: "RoadVisionEngine", frames, ts, depth: int = 2,
                 chunk: Optional[int] = None, capture: bool = True):
        """capture=False runs the same multi-stream schedule eagerly, right
        here (no graphs; run() is then a no-op): bench.py's per-launch conv
        timing uses it, since HIP events recorded inside captured graphs
        do not time on ROCm 7.2 (measured: zero elapsed).

        With a detector of L >= 2 forward lanes (RoadVisionEngine(lanes=L))
        the schedule is a dependency graph instead of lock-stepped stages:
        P(j) on one stream, Y(j) on lane stream j % L, T(j) on one stream;
        Y(j) waits for P(j) and for T(j - 2L) (its candidate slot), P(j) for
        Y(j - 2L) (its letterbox slot), T(j) for Y(j) -- so the forwards of
        L consecutive steps run concurrently while P runs ahead and T
        follows; SORT still sees every stream's frames in order (the T
        stages are one stream).  Each stage is its own captured graph and
        run() replays them chained by HIP events (_issue); `chunk` does not
        apply."""
        self.eng = eng
        if eng.pair > 1 and depth != 4:
            raise ValueError("RoadVisionEngine(pair > 1) runs the depth-4 pipeline only")
        ctx = (lambda g: torch.cuda.graph(g)) if capture else (lambda g: contextlib.nullcontext())
        K = len(frames)
        dev = eng.device
        side_t, side_p = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        self.graphs = []
        self.outs = []
        self.records = [Record(eng.S, eng.detector.max_det, dev) for _ in range(K)]
        procs = {}
        L = eng.detector.lanes
        slots = eng.detector.slots

        def track(j):
            o = eng.track_stage(ts[j], j % slots, self.records[j])
            return {"record": o["record"]}
        if chunk is None:  # default: 8 steps per graph (pair mode: 8 // pair units)
            chunk = int(os.environ.get("RV_GRAPH_CHUNK", "8"))
            if chunk > 0 and eng.pair > 1:
                chunk = max(1, chunk // eng.pair)
        self.staged = L > 1 and depth != 4
        if self.staged:
            # Per-stage graphs chained by events at replay time (run()): a
            # forward captured on a side stream of a multi-stream capture
            # crashes hipStreamEndCapture on ROCm 7.2 (tools/probe_lanes.py),
            # so every stage is captured alone on the capture stream and the
            # dependency graph lives in the replay order + HIP events.
            self.ys = [torch.cuda.Stream(dev) for _ in range(L)]
            self.side_p, self.side_t = side_p, side_t
            self.L, self.slots, self.K = L, slots, K
            mk = (lambda: torch.cuda.Event()) if capture else (lambda: None)
            self.eP = [mk() for _ in range(K)]
            self.eY = [mk() for _ in range(K)]
            self.eT = [mk() for _ in range(K)]
            self.gP, self.gY, self.gT = [], [], []
            if not capture:  # eager: the same chain, issued right here
                self._issue(lambda j: eng.preprocess_stage(frames[j], j % slots),
                            lambda j, lb: eng.yolo_stage(lb, j % slots, j % L),
                            track, procs, events=False)
                return
            for j in range(K):
                gp, gy, gt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gp):
                    procs[j], lb = eng.preprocess_stage(frames[j], j % slots)
                with torch.cuda.graph(gy):
                    eng.yolo_stage(lb, j % slots, j % L)
                with torch.cuda.graph(gt):
                    out = track(j)
                out["proc"] = procs.pop(j)
                self.outs.append(out)
                self.gP.append(gp)
                self.gY.append(gy)
                self.gT.append(gt)
            return
        if depth == 2:
            for j in range(K + 1):
                g = torch.cuda.CUDAGraph() if capture else None
                with ctx(g):
                    cur = torch.cuda.current_stream()
                    if j > 0:
                        side_t.wait_stream(cur)
                        with torch.cuda.stream(side_t):
                            out = track(j - 1)
                    if j < K:
                        procs[j], lb = eng.preprocess_stage(frames[j])
                    if j > 0:
                        cur.wait_stream(side_t)
                        out["proc"] = procs.pop(j - 1)
                        self.outs.append(out)
                    if j < K:
                        eng.yolo_stage(lb, j % 2)
                if capture:
                    self.graphs.append(g)
            return
        lbs = {}
        if depth == 4:
            self._capture_depth4(frames, ts, track, procs, lbs, chunk, ctx, capture)
            return
        # steps per captured graph (`chunk`, RV_GRAPH_CHUNK): consecutive
        # pipeline stages j are captured into one graph, so the device never
        # idles between graph replays inside a chunk; 0 = all K+2 stages in
        # one graph.  A serving loop replays one chunk per `chunk` steps.
        js = list(range(-1, K + 1))
        size = len(js) if chunk <= 0 else chunk
        for c0 in range(0, len(js), size):
            g = torch.cuda.CUDAGraph() if capture else None
            with ctx(g):
                for j in js[c0:c0 + size]:
                    cur = torch.cuda.current_stream()
                    side_t.wait_stream(cur)
                    side_p.wait_stream(cur)
                    if j + 1 < K:  # P(j+1) into letterbox slot (j+1) % 2
                        with torch.cuda.stream(side_p):
                            procs[j + 1], lbs[j + 1] = eng.preprocess_stage(frames[j + 1],
                                                                            (j + 1) % 2)
                    if j >= 1:  # T(j-1) from candidate slot (j-1) % 2
                        with torch.cuda.stream(side_t):
                            out = track(j - 1)
                    if 0 <= j < K:  # Y(j)
                        eng.yolo_stage(lbs.pop(j), j % 2)
                    cur.wait_stream(side_p)
                    cur.wait_stream(side_t)
                    if j >= 1:
                        out["proc"] = procs.pop(j - 1)
                        self.outs.append(out)
            if capture:
                self.graphs.append(g)

    def _capture_depth4(self, frames, ts, track, procs, lbs, chunk, ctx, capture):
        """depth=4 with two forward lanes: the forward is split in two
        (rv_yolo_forward_part) and stage j runs
            P(j+1) || Y1(j) || Y2(j-1) || T(j-2)
        -- the bandwidth-heavy first half of step j's forward beside the
        latency-bound second half of step j-1's (each step's forward uses
        lane j % 2: its own workspace), the preprocess of step j+1 and the
        NMS + SORT of step j-2.  Y2 runs on the capture stream (it forks the
        Detect heads); Y1, P and T on side streams."""
        eng = self.eng
        if eng.detector.lanes != 2:
            raise ValueError("depth 4 needs RoadVisionEngine(lanes=2)")
        P = eng.pair
        if len(frames) % P:
            raise ValueError(f"pair mode: the step count {len(frames)} is not a multiple of {P}")
        K = len(frames) // P  # pipeline units: P consecutive steps, one forward
        dev = eng.device
        side_p, side_t, side_y = (torch.cuda.Stream(dev) for _ in range(3))
        slots = eng.detector.slots
        S = eng.S
        if P > 1:  # a unit's stages over its P steps
            def prep(u, slot):
                for h in range(P):
                    procs[u * P + h], _ = eng.preprocess_stage(frames[u * P + h], slot, h * S)
                return None, eng.detector.lb[slot][:P * S]

            def trk(u, slot):
                return eng.track_pair_stage([ts[u * P + h] for h in range(P)], slot,
                                            [self.records[u * P + h] for h in range(P)])
        js = list(range(-1, K + 2))
        size = len(js) if chunk <= 0 else chunk
        for c0 in range(0, len(js), size):
            g = torch.cuda.CUDAGraph() if capture else None
            with ctx(g):
                for j in js[c0:c0 + size]:
                    cur = torch.cuda.current_stream()
                    for x in (side_p, side_t, side_y):
                        x.wait_stream(cur)
                    res = {}

                    def p_(j=j):  # P(j+1) into letterbox slot (j+1) % slots
                        if 0 <= j + 1 < K:
                            with torch.cuda.stream(side_p):
                                if P > 1:
                                    _, lbs[j + 1] = prep(j + 1, (j + 1) % slots)
                                else:
                                    procs[j + 1], lbs[j + 1] = eng.preprocess_stage(
                                        frames[j + 1], (j + 1) % slots)

                    def t_(j=j):  # T(j-2) from candidate slot (j-2) % slots
                        if 0 <= j - 2 < K:
                            with torch.cuda.stream(side_t):
                                res["out"] = (trk(j - 2, (j - 2) % slots) if P > 1
                                              else track(j - 2))

                    def y1_(j=j):  # Y1(j) on lane j % 2
                        if 0 <= j < K:
                            with torch.cuda.stream(side_y):
                                eng.yolo_stage(lbs.pop(j), j % slots, j % 2, part=1)

                    def y2_(j=j):  # Y2(j-1): candidates into slot (j-1) % slots
                        if 0 <= j - 1 < K:
                            eng.yolo_stage(None, (j - 1) % slots, (j - 1) % 2, part=2)
                    # capture order = the graph executor's launch order, which
                    # decides which HW queue a branch lands on and what it
                    # queues behind: Y2, P, Y1, T measured best (tools: the
                    # DESIGN.md schedule table; Y1 before P costs 10 %)
                    y2_()
                    p_()
                    y1_()
                    t_()
                    out = res.get("out")
                    for x in (side_p, side_t, side_y):
                        cur.wait_stream(x)
                    if 0 <= j - 2 < K:
                        for h, o in enumerate(out if P > 1 else [out]):
                            o["proc"] = procs.pop((j - 2) * P + h)
                            self.outs.append(o)
            if capture:
                self.graphs.append(g)

    def _issue(self, P, Y, T, procs=None, events=True):
        """The multi-lane chain: P(j) on side_p after Y(j - slots) (its
        letterbox slot), Y(j) on lane stream j % L after P(j) and T(j - slots)
        (its candidate slot), T(j) on side_t after Y(j); SORT sees the T's in
        step order.  With graphs P / Y / T replay the captured stages; eager
        (events=False) they run the stage functions and use fresh events."""
        cur = torch.cuda.current_stream()
        sp, st, ys = self.side_p, self.side_t, self.ys
        for x in [sp, st] + ys:
            x.wait_stream(cur)
        eP, eY, eT = ((self.eP, self.eY, self.eT) if events else
                      ([torch.cuda.Event() for _ in range(self.K)] for _ in range(3)))
        S = self.slots
        lbs = {}
        for j in range(self.K):
            ln = ys[j % self.L]
            with torch.cuda.stream(sp):
                if j >= S:
                    sp.wait_event(eY[j - S])
                r = P(j)
                if procs is not None:
                    procs[j], lbs[j] = r
                eP[j].record(sp)
            with torch.cuda.stream(ln):
                ln.wait_event(eP[j])
                if j >= S:
                    ln.wait_event(eT[j - S])
                Y(j, lbs.pop(j, None))
                eY[j].record(ln)
            with torch.cuda.stream(st):
                st.wait_event(eY[j])
                out = T(j)
                eT[j].record(st)
            if procs is not None:
                out["proc"] = procs.pop(j)
                self.outs.append(out)
        for x in [sp, st] + ys:
            cur.wait_stream(x)

    def run(self):
        if self.staged:
            if self.gP:
                self._issue(lambda j: self.gP[j].replay(), lambda j, lb: self.gY[j].replay(),
                            lambda j: self.gT[j].replay())
            return
        for g in self.graphs:
            g.replay()
