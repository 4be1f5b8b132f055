"""HIP YOLOv8 detector backend (drop-in for src/detect/yolo_ultralytics.py).

``YoloEngine`` is the batched device path: letterbox (rv_letterbox_u8) ->
YOLOv8 forward on MFMA with fused decode/candidate filter (rv_yolo_forward) ->
batched NMS + scale_boxes + class filter (rv_nms_postprocess).  Everything
stays on the GPU; only ``to_detections`` copies the (B, max_det, 6) result to
the host to build ``Detection`` objects, matching yolo_ultralytics.py:44-52.

``YOLOHip`` wraps it behind the reference's ``Detector`` interface with the
same config keys (model, device, conf_thres, iou_thres, max_det,
classes_keep; yolo_ultralytics.py:15-24).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import _lib, kernels
from .._lib import call, ptr, stream_ptr
from .base import Detector
from .types import Detection
from .weights import COCO80, DTYPES, pack, variant_of, weights_from_config

CAND_BYTES = 32


def scale_boxes_params(img1_hw, img0_hw):
    """Ultralytics ops.scale_boxes(img1_shape, boxes, img0_shape) constants:
    (gain, pad_x, pad_y) with python-float gain and python round()."""
    gain = min(img1_hw[0] / img0_hw[0], img1_hw[1] / img0_hw[1])
    pad_x = round((img1_hw[1] - img0_hw[1] * gain) / 2 - 0.1)
    pad_y = round((img1_hw[0] - img0_hw[0] * gain) / 2 - 0.1)
    return gain, pad_x, pad_y


def class_mask(classes_keep: Sequence[int]) -> Optional[np.ndarray]:
    keep = set(int(x) for x in classes_keep)
    if not keep:
        return None
    m = np.zeros(4, np.uint32)
    for c in keep:
        if 0 <= c < 128:
            m[c >> 5] |= np.uint32(1 << (c & 31))
    return m


class YoloEngine:
    """Batched letterbox -> YOLOv8 -> NMS for frames of one (H, W).

    `lanes` > 1 keeps that many independent forward contexts (plan handle +
    activation workspace; the packed weights are shared), so forwards of
    consecutive steps can run concurrently on different HIP streams -- each
    forward is a latency-bound chain of small launches that leaves most of
    the chip idle.  Letterbox and candidate buffers have 2 * lanes slots.

    dtype 'fp8' (BASELINE configs[4]): the conv stack runs on the fp8 MFMA
    (OCP e4m3 weights and activations, power-of-two scales; include/rvhip.h
    RV_YOLO_DTYPE_FP8).  Its per-buffer activation scales come from
    `act_scales` (a saved calibration) or from calibrate(); a forward before
    either raises."""

    def __init__(self, variant: int, flat_weights: np.ndarray, max_batch: int, frame_hw,
                 imgsz: int = 640, stride: int = 32, conf: float = 0.25, iou: float = 0.7,
                 max_det: int = 100, classes_keep: Sequence[int] = (), max_wh: float = 7680.0,
                 max_nms: int = 30000, device="cuda", lanes: int = 1, dtype: str = "bf16",
                 act_scales: Optional[Sequence[float]] = None):
        self.device = torch.device(device)
        self.variant = variant
        if dtype not in DTYPES:
            raise ValueError(f"dtype {dtype!r}: expected one of {sorted(DTYPES)}")
        self.dtype = dtype
        self.flat = flat_weights
        self.H, self.W = int(frame_hw[0]), int(frame_hw[1])
        self.max_batch = int(max_batch)
        self.conf, self.iou, self.max_det, self.max_wh = float(conf), float(iou), int(max_det), \
            float(max_wh)
        self.max_nms = int(max_nms)  # Ultralytics non_max_suppression default
        self.geo = kernels.letterbox_geometry(self.H, self.W, imgsz, stride)
        self.in_h, self.in_w = self.geo[0], self.geo[1]
        self.packed = torch.from_numpy(pack(variant, flat_weights, dtype)).to(self.device)
        self.lanes = max(1, int(lanes))
        self._hs = []
        for _ in range(self.lanes):
            h = ctypes.c_void_p()
            call("rv_yolo_create2", variant, DTYPES[dtype], ptr(self.packed), self.max_batch,
                 self.in_h, self.in_w, ctypes.byref(h))
            self._hs.append(h)
        self._h = h = self._hs[0]
        lib = _lib.load()
        self.A = lib.rv_yolo_num_anchors(h)
        self.nc = 80
        self.ws_bytes = lib.rv_yolo_ws_bytes(h, self.max_batch)
        dev = self.device
        self.wss = [torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
                    for _ in range(self.lanes)]
        self.ws = self.wss[0]
        self.slots = 2 * self.lanes
        # letterbox slots: a pipelined engine letterboxes frame k+1 while the
        # forward(s) of earlier frames still read theirs
        self.lb = torch.empty((self.slots, self.max_batch, self.in_h, self.in_w, 3),
                              dtype=torch.uint8, device=dev)
        # segmented candidate layout: nseg segments of 64 rows per image
        self.nseg = lib.rv_yolo_cand_segments(h)
        self.cap = 64 * max(self.nseg, lib.rv_cand_segments(self.A))
        # candidate slots: a pipelined engine decodes frame k+1 into one slot
        # while NMS still reads frame k's from another
        self.cand = torch.empty((self.slots, self.max_batch, self.cap, CAND_BYTES // 4),
                                dtype=torch.float32, device=dev)
        self.seg_n = torch.zeros((self.slots, self.max_batch,
                                  max(self.nseg, lib.rv_cand_segments(self.A))),
                                 dtype=torch.int32, device=dev)
        # NMS outputs and workspace (sort keys of images with more than 4096
        # candidates) per candidate slot: a pipelined engine runs unit u's NMS
        # beside the SORT steps of unit u-1 (rvs_amd.schedule); the
        # unsuffixed names are slot 0's
        self.cand_n_s = torch.zeros((self.slots, self.max_batch), dtype=torch.int32, device=dev)
        self.nms_ws_s = torch.empty((self.slots, max(int(_lib.load().rv_nms_ws_bytes(self.max_batch)), 8)),
                                    dtype=torch.uint8, device=dev)
        self._nseg_cur = self.nseg
        self.dets_s = torch.zeros((self.slots, self.max_batch, self.max_det, 6), dtype=torch.float32,
                                  device=dev)
        self.det_n_s = torch.zeros((self.slots, self.max_batch), dtype=torch.int32, device=dev)
        self.cand_n, self.nms_ws = self.cand_n_s[0], self.nms_ws_s[0]
        self.dets, self.det_n = self.dets_s[0], self.det_n_s[0]
        gain, px, py = scale_boxes_params((self.in_h, self.in_w), (self.H, self.W))
        self.scale5 = torch.tensor([gain, px, py, self.W, self.H], dtype=torch.float32, device=dev)
        m = class_mask(classes_keep)
        self.keep = None if m is None else torch.from_numpy(m.view(np.int32)).to(dev)
        self.act_scales = None
        if act_scales is not None:
            self.set_act_scales(act_scales)

    def buffers(self, B: int, h=None):
        """Activation buffers of the plan for batch B: [(name, H, W, C,
        element bytes, byte offset in the workspace)]."""
        lib = _lib.load()
        h = self._h if h is None else h
        out = []
        for i in range(lib.rv_yolo_num_buffers(h)):
            info = (ctypes.c_int * 4)()
            off = ctypes.c_size_t()
            call("rv_yolo_buffer_info", h, B, i, info, ctypes.byref(off))
            name = ctypes.create_string_buffer(64)
            call("rv_yolo_buffer_name", h, i, name, 64)
            out.append((name.value.decode(), info[0], info[1], info[2],
                        lib.rv_yolo_buffer_esize(h, i), off.value))
        return out

    def set_act_scales(self, scales: Sequence[float]) -> None:
        """Per-buffer fp8 activation scales (powers of two; the order of
        buffers())."""
        arr = (ctypes.c_float * len(scales))(*[float(x) for x in scales])
        for h in self._hs:
            call("rv_yolo_set_act_scales", h, arr, len(scales))
        self.act_scales = [float(x) for x in scales]

    def calibrate(self, lb: torch.Tensor) -> List[float]:
        """fp8 plans: one power-of-two scale per activation buffer, from the
        absolute maximum the bf16 plan of the same weights reaches in that
        buffer on this letterboxed batch (rv_fp8_scale: amax / scale in
        (224, 448]); installs and returns them."""
        lib = _lib.load()
        B = lb.shape[0]
        packed = torch.from_numpy(pack(self.variant, self.flat, "bf16")).to(self.device)
        h = ctypes.c_void_p()
        call("rv_yolo_create2", self.variant, 0, ptr(packed), B, self.in_h, self.in_w,
             ctypes.byref(h))
        try:
            ws = torch.empty(lib.rv_yolo_ws_bytes(h, B), dtype=torch.uint8, device=self.device)
            raw = torch.empty((B, 4 + self.nc, self.A), dtype=torch.float32, device=self.device)
            # raw forward with RV_YOLO_OPT_RAW_UNFUSED (default): every buffer written
            call("rv_yolo_forward", h, ptr(lb.contiguous()), B, ptr(ws), ws.numel(), ptr(raw),
                 self.conf, None, 0, None, stream_ptr())
            scales = []
            for name, H, W, C, es, off in self.buffers(B, h):
                n = B * H * W * C
                v = ws[off:off + n * es].view(torch.float32 if es == 4 else torch.bfloat16)
                amax = float(v.float().abs().max().item()) if n else 0.0
                scales.append(float(lib.rv_fp8_scale(amax)))
            torch.cuda.synchronize(self.device)
        finally:
            lib.rv_yolo_destroy(h)
        self.set_act_scales(scales)
        return scales

    def close(self):
        for h in getattr(self, "_hs", []):
            if h:
                _lib.load().rv_yolo_destroy(h)
        self._hs = []
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_raw_fused(self, fused: bool) -> None:
        """Raw forwards run the production kernel sequence (fused stem) when
        True, so forward_raw(raw) reproduces the candidate path's prediction
        exactly; False (default) keeps every activation for layer tests."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 1, 0 if fused else 1)

    def set_stem_x1(self, on: bool) -> None:
        """The fused stem also writes the X1 map (RV_YOLO_OPT_STEM_X1; by
        default X1 stays in registers when model.2.cv1 is fused into it)."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 3, 1 if on else 0)

    def set_head_streams(self, on: bool) -> None:
        """The P3 / P4 Detect heads on the handle's two side streams (True,
        default) or on the caller's stream (RV_YOLO_OPT_HEAD_STREAMS)."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 4, 1 if on else 0)

    def set_fuse_cv1(self, on: bool) -> None:
        """model.3 and model.4.cv1 as one launch with the 1x1 chained on
        model.3's output tile in LDS (True, default) or as two launches
        (RV_YOLO_OPT_FUSE_CV1; bit-identical results)."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 5, 1 if on else 0)

    def set_head_chain(self, on: bool) -> None:
        """Candidate forwards run each Detect branch's last 1x1 conv inside
        its 3x3 conv's launch plus one small combine kernel (True)
        or through the decode kernel (RV_YOLO_OPT_HEAD_CHAIN; the same
        candidates; off by default)."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 6, 1 if on else 0)

    def set_c2f_tap_pairs(self, on: bool) -> None:
        """The fused width-16 C2f chain's 3x3 convs on tap pairs (True,
        default: within 1 bf16 ulp of the per-tap k order) or one k-step per
        tap (False: bit-identical to the unfused launches;
        RV_YOLO_OPT_C2F_TAP_PAIRS)."""
        for h in self._hs:
            call("rv_yolo_set_option", h, 7, 1 if on else 0)

    def set_fuse_c2f(self, on) -> None:
        """Narrow C2f blocks as one fused launch or one launch per conv
        (RV_YOLO_OPT_FUSE_C2F; bit-identical results): True / 1 = the
        hidden-width-16 chains only (default), 2 = widths 16 and 32,
        False / 0 = none."""
        v = 1 if on is True else (0 if on is False else int(on))
        for h in self._hs:
            call("rv_yolo_set_option", h, 2, v)

    def letterbox(self, frames: torch.Tensor, slot: int = 0, off: int = 0) -> torch.Tensor:
        """Letterbox into images [off, off + B) of letterbox slot `slot`."""
        B = frames.shape[0]
        return kernels.letterbox(frames, self.geo, out=self.lb[slot][off:off + B])

    def forward_raw(self, lb: Optional[torch.Tensor], raw: Optional[torch.Tensor] = None,
                    candidates: bool = True, slot: int = 0, lane: int = 0, part: int = 0,
                    batch: Optional[int] = None):
        """YOLOv8 forward + decode in forward context `lane`; candidates go to
        candidate slot `slot`.  part 1 / 2: the two halves of the forward
        (rv_yolo_forward_part; part 2 takes no letterbox, `batch` gives B)."""
        B = lb.shape[0] if lb is not None else int(batch)
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        if lb is not None:
            lb = lb.contiguous()
        call("rv_yolo_forward_part", self._hs[lane], ptr(lb), B, ptr(self.wss[lane]),
             self.ws_bytes, ptr(raw), self.conf, ptr(self.cand[slot]) if candidates else None,
             self.cap, ptr(self.seg_n[slot]) if candidates else None, stream_ptr(), int(part))
        self._nseg_cur = self.nseg
        return raw

    def autotune(self, lb: torch.Tensor, reps: int = 3, verify: bool = False) -> int:
        """Pick the fastest kernel configuration of every conv launch on this
        letterboxed batch (rv_yolo_autotune; synchronous, not capturable).
        Returns the number of configurations whose output differed from the
        default's (verify=True; 0 expected: all are bit-identical)."""
        B = lb.shape[0]
        lb = lb.contiguous()
        bad = ctypes.c_int(0)
        call("rv_yolo_autotune", self._h, ptr(lb), B, ptr(self.ws), self.ws_bytes, int(reps),
             1 if verify else 0, ctypes.byref(bad), stream_ptr())
        if self.lanes > 1:  # the other forward contexts run the same plan
            cfgs = self.tuned_configs()
            for h in self._hs[1:]:
                for i, c in enumerate(cfgs):
                    call("rv_yolo_set_tuned", h, len(cfgs), i, _lib.int_array(c))
        return bad.value

    def tuned_configs(self):
        """[(MR, NR, G, resw, persist, kind)] per conv launch ([] before autotune)."""
        lib = _lib.load()
        n = lib.rv_yolo_tuned_config(self._h, -1, None)
        out = []
        for i in range(max(n, 0)):
            c = (ctypes.c_int * 6)()
            lib.rv_yolo_tuned_config(self._h, i, c)
            out.append(tuple(c))
        return out

    def conv_candidates(self, idx: int):
        """Valid (MR, NR, G, resw, persist, kind) configurations of conv
        launch idx of the last whole forward of lane 0 ([] for a fused C2f
        launch)."""
        n = call("rv_yolo_conv_candidates", self._h, int(idx), None, 0)
        if n < 0:
            _lib.check(n, "rv_yolo_conv_candidates")
        buf = (ctypes.c_int * (6 * max(n, 1)))()
        call("rv_yolo_conv_candidates", self._h, int(idx), buf, n)
        return [tuple(buf[6 * i:6 * i + 6]) for i in range(n)]

    def load_tuned(self, cfgs) -> None:
        """Install saved per-launch configurations (tuned_configs() of an
        earlier autotune of the same plan) instead of autotuning."""
        n = len(cfgs)
        for h in self._hs:
            for i, c in enumerate(cfgs):
                call("rv_yolo_set_tuned", h, n, i, _lib.int_array(c))

    def nms(self, B: int, slot: int = 0):
        """NMS + scale_boxes + class filter of candidate slot `slot`, into
        that slot's outputs."""
        call("rv_nms_postprocess", ptr(self.cand[slot]), ptr(self.seg_n[slot]), B, self.cap,
             self._nseg_cur, self.iou, self.max_det, self.max_nms, self.max_wh, ptr(self.scale5),
             ptr(self.keep),
             ptr(self.dets_s[slot]), ptr(self.det_n_s[slot]), ptr(self.cand_n_s[slot]),
             ptr(self.nms_ws_s[slot]), self.nms_ws_s[slot].numel(), stream_ptr())
        return self.dets_s[slot][:B], self.det_n_s[slot][:B]

    def nms_from_raw(self, raw: torch.Tensor):
        """Reference-layout entry (B, 4+nc, A) -> NMS (parity tests)."""
        B, C, A = raw.shape
        raw = raw.contiguous()
        if self.seg_n[0].numel() < B * _lib.load().rv_cand_segments(A) or \
                self.cap < 64 * _lib.load().rv_cand_segments(A):
            raise ValueError(f"raw prediction with A={A} exceeds the candidate buffers")
        self._nseg_cur = _lib.load().rv_cand_segments(A)
        seg = self.seg_n[0].view(-1)[:B * self._nseg_cur].view(B, self._nseg_cur)
        call("rv_candidates_from_raw", ptr(raw), B, C - 4, A, self.conf, ptr(self.cand[0]),
             self.cap, ptr(seg), stream_ptr())
        return self.nms(B)

    def run(self, frames: torch.Tensor):
        """(B,H,W,3) u8 device frames -> (dets (B,max_det,6), counts (B,)) on device."""
        if frames.dim() == 3:
            frames = frames.unsqueeze(0)
        B = frames.shape[0]
        self.forward_raw(self.letterbox(frames))
        return self.nms(B)

    def run_letterboxed(self, lb: torch.Tensor):
        """Already letterboxed (B,in_h,in_w,3) u8 device batch -> (dets, counts)."""
        self.forward_raw(lb)
        return self.nms(lb.shape[0])

    @staticmethod
    def to_detections(dets: torch.Tensor, det_n: torch.Tensor, names=COCO80) -> List[List[Detection]]:
        d = dets.cpu().numpy()
        n = det_n.cpu().numpy()
        out = []
        for b in range(d.shape[0]):
            lst = []
            for r in d[b, :int(n[b])]:
                k = int(r[5])
                name = str(names[k]) if names is not None and 0 <= k < len(names) else str(k)
                lst.append(Detection(float(r[0]), float(r[1]), float(r[2]), float(r[3]),
                                     float(r[4]), k, name))
            out.append(lst)
        return out


class YOLOHip(Detector):
    """Config-compatible replacement of YOLOUltralytics (backend 'hip')."""

    def __init__(self, cfg: Dict):
        device = cfg.get("device", "auto")
        self.device = torch.device("cuda:0" if device in ("auto", None, "cpu") else device)
        if not torch.cuda.is_available():
            raise RuntimeError("YOLOHip needs an MI355X (HIP device); there is no CPU fallback")
        self.variant = variant_of(cfg.get("model", "yolov8n.pt"))
        self.flat = weights_from_config(cfg, self.variant)
        self.conf = float(cfg.get("conf_thres", 0.25))
        self.iou = float(cfg.get("iou_thres", 0.7))
        self.max_det = int(cfg.get("max_det", 100))
        self.keep = [int(x) for x in cfg.get("classes_keep", [])]
        self.imgsz = int(cfg.get("imgsz", 640))
        self.names = COCO80
        self._engines: Dict = {}

    def engine(self, H: int, W: int, max_batch: int = 1) -> YoloEngine:
        key = (H, W)
        e = self._engines.get(key)
        if e is None or e.max_batch < max_batch:
            if e is not None:  # a larger batch replaces it: free its plan first
                e.close()
            e = YoloEngine(self.variant, self.flat, max_batch, (H, W), imgsz=self.imgsz,
                           conf=self.conf, iou=self.iou, max_det=self.max_det,
                           classes_keep=self.keep, device=self.device)
            self._engines[key] = e
        return e

    def infer_batch(self, frames: torch.Tensor) -> List[List[Detection]]:
        if frames.dim() == 3:
            frames = frames.unsqueeze(0)
        eng = self.engine(frames.shape[1], frames.shape[2], frames.shape[0])
        dets, n = eng.run(frames)
        return YoloEngine.to_detections(dets, n, self.names)

    def infer(self, bgr) -> List[Detection]:
        if isinstance(bgr, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(bgr)).to(self.device)
        else:
            x = bgr
        return self.infer_batch(x)[0]

    def close(self):
        for e in self._engines.values():
            e.close()
        self._engines.clear()
