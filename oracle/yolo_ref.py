"""Torch-CPU fp32 restatement of the detector path -- TEST INFRASTRUCTURE ONLY.

Restates what src/detect/yolo_ultralytics.py:26-53 gets from Ultralytics
(~8.3.x, absent here; parity vs real Ultralytics is UNPINNED, and no trained
weights exist in this environment):
  * the yolov8.yaml graph: Conv(conv+BN(fused)+SiLU), C2f, SPPF, nearest
    Upsample, Concat, Detect (DFL softmax expectation, dist2bbox xywh *
    stride, class sigmoid); written here independently of the HIP plan so the
    two restatements check each other;
  * predictor preprocess: BGR->RGB, HWC->CHW, float32 / 255;
  * non_max_suppression (agnostic=False, max_wh=7680, max_nms=30000) with
    torchvision.ops.nms semantics (oracle C: oracle_nms), scale_boxes, and the
    reference's post-NMS classes_keep filter (yolo_ultralytics.py:49-50).
Weights come in as the flat f32 array of rvs weights (per conv, in
Ultralytics state_dict order: weight[cout][cin][k][k], bias[cout]).
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import cpu

SCALES = {0: (0.33, 0.25, 1024), 1: (0.33, 0.50, 1024), 2: (0.67, 0.75, 768),
          3: (1.00, 1.00, 512), 4: (1.00, 1.25, 512)}


def _ch(c, w, mc):
    return int(math.ceil(min(c, mc) * w / 8) * 8)


def conv_specs(variant: int):
    """[(name, cin, cout, k, s, silu)] in Ultralytics state_dict order."""
    d, w, mc = SCALES[variant]
    ch = lambda c: _ch(c, w, mc)  # noqa: E731
    rep = lambda n: max(round(n * d), 1)  # noqa: E731
    specs = []

    def conv(n, ci, co, k, s, act=1):
        specs.append((n, ci, co, k, s, act))

    def c2f(p, c1, c2, n):
        c = c2 // 2
        conv(p + ".cv1", c1, 2 * c, 1, 1)
        conv(p + ".cv2", (2 + n) * c, c2, 1, 1)
        for i in range(n):
            conv(f"{p}.m.{i}.cv1", c, c, 3, 1)
            conv(f"{p}.m.{i}.cv2", c, c, 3, 1)

    c1, c2, c3, c4, c5 = ch(64), ch(128), ch(256), ch(512), ch(1024)
    h12, h15, h18, h21 = ch(512), ch(256), ch(512), ch(1024)
    nb, nm = rep(3), rep(6)
    conv("model.0", 3, c1, 3, 2)
    conv("model.1", c1, c2, 3, 2)
    c2f("model.2", c2, c2, nb)
    conv("model.3", c2, c3, 3, 2)
    c2f("model.4", c3, c3, nm)
    conv("model.5", c3, c4, 3, 2)
    c2f("model.6", c4, c4, nm)
    conv("model.7", c4, c5, 3, 2)
    c2f("model.8", c5, c5, nb)
    conv("model.9.cv1", c5, c5 // 2, 1, 1)
    conv("model.9.cv2", c5 // 2 * 4, c5, 1, 1)
    c2f("model.12", c5 + c4, h12, nb)
    c2f("model.15", h12 + c3, h15, nb)
    conv("model.16", h15, h15, 3, 2)
    c2f("model.18", h15 + h12, h18, nb)
    conv("model.19", h18, h18, 3, 2)
    c2f("model.21", h18 + c5, h21, nb)
    chs = (h15, h18, h21)
    c2d = max(16, h15 // 4, 64)
    c3d = max(h15, min(80, 100))
    for i in range(3):
        conv(f"model.22.cv2.{i}.0", chs[i], c2d, 3, 1)
        conv(f"model.22.cv2.{i}.1", c2d, c2d, 3, 1)
        conv(f"model.22.cv2.{i}.2", c2d, 64, 1, 1, 0)
    for i in range(3):
        conv(f"model.22.cv3.{i}.0", chs[i], c3d, 3, 1)
        conv(f"model.22.cv3.{i}.1", c3d, c3d, 3, 1)
        conv(f"model.22.cv3.{i}.2", c3d, 80, 1, 1, 0)
    meta = dict(nb=nb, nm=nm)
    return specs, meta


def _bf16(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


class YoloRef:
    """fp32 CPU forward of YOLOv8 from flat fused weights.

    quant=True emulates the HIP path's storage precision (bf16 weights except
    the first conv, bf16 activations rounded once after bias/SiLU/residual,
    f32 head logits) with f32 accumulation, to separate kernel errors from
    quantisation effects in the parity tests."""

    def __init__(self, variant: int, flat: np.ndarray, quant: bool = False):
        self.quant = quant
        self.specs, meta = conv_specs(variant)
        self.nb, self.nm = meta["nb"], meta["nm"]
        self.p = {}
        off = 0
        flat = np.asarray(flat, np.float32)
        for n, ci, co, k, s, act in self.specs:
            nw = co * ci * k * k
            w = torch.from_numpy(flat[off:off + nw].reshape(co, ci, k, k).copy())
            b = torch.from_numpy(flat[off + nw:off + nw + co].copy())
            off += nw + co
            if quant and n != "model.0":
                w = _bf16(w)
            self.p[n] = (w, b, s, k, act)
        assert off == flat.size, "flat weight size mismatch"
        self.bn = {}

    @classmethod
    def from_unfused(cls, variant: int, sd: dict, eps: float = 1e-3) -> "YoloRef":
        """The UNFUSED Ultralytics network of a state_dict (Conv = conv2d
        without bias -> BatchNorm2d(eps) in eval mode -> SiLU; the Detect
        head's last convs plain conv2d + bias): what model.fuse()
        (yolo_ultralytics.py:16-17) replaces by folded convs."""
        specs, _ = conv_specs(variant)
        flat = []
        for n, ci, co, k, s, act in specs:
            key = n + ".conv.weight" if n + ".conv.weight" in sd else n + ".weight"
            flat += [np.asarray(sd[key], np.float32).ravel(),
                     np.asarray(sd.get(n + ".bias", np.zeros(co)), np.float32).ravel()]
        m = cls(variant, np.concatenate(flat))
        for n, ci, co, k, s, act in specs:
            if n + ".bn.running_var" in sd:
                t = lambda x: torch.from_numpy(np.asarray(sd[n + x], np.float32))  # noqa: E731
                m.bn[n] = (t(".bn.running_mean"), t(".bn.running_var"), t(".bn.weight"),
                           t(".bn.bias"), eps)
        return m

    def conv(self, n, x, res=None):
        w, b, s, k, act = self.p[n]
        if n in self.bn:
            mean, var, g, beta, eps = self.bn[n]
            y = F.batch_norm(F.conv2d(x, w, None, stride=s, padding=k // 2), mean, var, g, beta,
                             False, 0.0, eps)
        else:
            y = F.conv2d(x, w, b, stride=s, padding=k // 2)
        y = F.silu(y) if act else y
        if res is not None:
            y = res + y
        if self.quant and not (n.startswith("model.22.") and n.endswith(".2")):
            y = _bf16(y)
        return y

    def c2f(self, p, x, n, shortcut):
        y = list(self.conv(p + ".cv1", x).chunk(2, 1))
        for i in range(n):
            t = y[-1]
            y.append(self.conv(f"{p}.m.{i}.cv2", self.conv(f"{p}.m.{i}.cv1", t),
                               res=t if shortcut else None))
        return self.conv(p + ".cv2", torch.cat(y, 1))

    def sppf(self, x):
        x = self.conv("model.9.cv1", x)
        y1 = F.max_pool2d(x, 5, 1, 2)
        y2 = F.max_pool2d(y1, 5, 1, 2)
        y3 = F.max_pool2d(y2, 5, 1, 2)
        return self.conv("model.9.cv2", torch.cat([x, y1, y2, y3], 1))

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B,3,H,W) f32 RGB in [0,1] -> raw (B, 84, A)."""
        up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")  # noqa: E731
        x = self.conv("model.0", x)
        x = self.conv("model.1", x)
        x = self.c2f("model.2", x, self.nb, True)
        x = self.conv("model.3", x)
        p4 = self.c2f("model.4", x, self.nm, True)
        x = self.conv("model.5", p4)
        p6 = self.c2f("model.6", x, self.nm, True)
        x = self.conv("model.7", p6)
        x = self.c2f("model.8", x, self.nb, True)
        p9 = self.sppf(x)
        p12 = self.c2f("model.12", torch.cat([up(p9), p6], 1), self.nb, False)
        p15 = self.c2f("model.15", torch.cat([up(p12), p4], 1), self.nb, False)
        p18 = self.c2f("model.18", torch.cat([self.conv("model.16", p15), p12], 1), self.nb, False)
        p21 = self.c2f("model.21", torch.cat([self.conv("model.19", p18), p9], 1), self.nb, False)
        feats = [p15, p18, p21]
        outs, anchors, strides = [], [], []
        for i, f in enumerate(feats):
            box = self.conv(f"model.22.cv2.{i}.2", self.conv(f"model.22.cv2.{i}.1",
                                                             self.conv(f"model.22.cv2.{i}.0", f)))
            cls = self.conv(f"model.22.cv3.{i}.2", self.conv(f"model.22.cv3.{i}.1",
                                                             self.conv(f"model.22.cv3.{i}.0", f)))
            outs.append(torch.cat([box, cls], 1).flatten(2))
            h, w = f.shape[2:]
            s = 8 * 2 ** i
            sy, sx = torch.meshgrid(torch.arange(h, dtype=torch.float32) + 0.5,
                                    torch.arange(w, dtype=torch.float32) + 0.5, indexing="ij")
            anchors.append(torch.stack([sx, sy], -1).view(-1, 2))
            strides.append(torch.full((h * w, 1), float(s)))
        y = torch.cat(outs, 2)
        anc = torch.cat(anchors).T.unsqueeze(0)
        st = torch.cat(strides).T
        B = y.shape[0]
        box, cls = y[:, :64], y[:, 64:]
        # DFL: softmax over 16 bins per side, expectation with arange(16)
        dist = (box.view(B, 4, 16, -1).softmax(2) *
                torch.arange(16, dtype=torch.float32).view(1, 1, 16, 1)).sum(2)
        lt, rb = dist.chunk(2, 1)
        x1y1 = anc - lt
        x2y2 = anc + rb
        dbox = torch.cat([(x1y1 + x2y2) / 2, x2y2 - x1y1], 1) * st
        return torch.cat([dbox, cls.sigmoid()], 1)


def preprocess(lb_bgr: np.ndarray) -> torch.Tensor:
    """Letterboxed BGR u8 (B,H,W,3) -> (B,3,H,W) f32 RGB / 255."""
    x = np.ascontiguousarray(lb_bgr[..., ::-1].transpose(0, 3, 1, 2))
    return torch.from_numpy(x).float() / 255


def scale_boxes_params(img1_hw, img0_hw):
    gain = min(img1_hw[0] / img0_hw[0], img1_hw[1] / img0_hw[1])
    pad = (round((img1_hw[1] - img0_hw[1] * gain) / 2 - 0.1),
           round((img1_hw[0] - img0_hw[0] * gain) / 2 - 0.1))
    return gain, pad


def postprocess(raw: np.ndarray, img1_hw, img0_hw, conf=0.25, iou=0.7, max_det=100,
                max_nms=30000, max_wh=7680.0, classes_keep: Sequence[int] = ()) -> List[np.ndarray]:
    """raw (B, 4+nc, A) f32 -> per image (n, 6) [x1,y1,x2,y2,conf,cls] (f32)."""
    raw = np.asarray(raw, np.float32)
    gain, pad = scale_boxes_params(img1_hw, img0_hw)
    keep_set = set(int(c) for c in classes_keep)
    out = []
    for r in raw:
        scores = r[4:]
        xc = scores.max(0) > np.float32(conf)
        x = r[:, xc].T  # (n, 84) in anchor order
        if x.shape[0] == 0:
            out.append(np.zeros((0, 6), np.float32))
            continue
        cx, cy, w, h = x[:, 0], x[:, 1], x[:, 2], x[:, 3]
        hw, hh = w / np.float32(2), h / np.float32(2)
        box = np.stack([cx - hw, cy - hh, cx + hw, cy + hh], 1).astype(np.float32)
        cls = x[:, 4:]
        j = cls.argmax(1)
        cf = cls[np.arange(len(j)), j]
        m = cf > np.float32(conf)
        box, cf, j = box[m], cf[m], j[m]
        if box.shape[0] > max_nms:
            o = np.argsort(-cf, kind="stable")[:max_nms]
            box, cf, j = box[o], cf[o], j[o]
        off = (j.astype(np.float32) * np.float32(max_wh))[:, None]
        keep = cpu.nms(box + off, cf, iou, max_det)
        rows = np.concatenate([box[keep], cf[keep, None], j[keep, None].astype(np.float32)], 1)
        rows = rows.astype(np.float32)
        rows[:, [0, 2]] -= np.float32(pad[0])
        rows[:, [1, 3]] -= np.float32(pad[1])
        rows[:, :4] /= np.float32(gain)
        rows[:, [0, 2]] = np.clip(rows[:, [0, 2]], 0, img0_hw[1])
        rows[:, [1, 3]] = np.clip(rows[:, [1, 3]], 0, img0_hw[0])
        if keep_set:
            rows = rows[[int(c) in keep_set for c in rows[:, 5]]]
        out.append(rows)
    return out
