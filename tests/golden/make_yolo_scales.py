"""Calibrate the synthetic YOLOv8 weights (data generation, run offline).

No trained checkpoint exists in this environment (yolov8n.pt is listed in the
reference's .MISSING_LARGE_BLOBS and there is no network).  A trained,
BN-fused YOLOv8 keeps every conv's pre-activation at O(1) scale; random
He-normal weights do not (activations vanish or explode through 60+ convs).
This script normalises every conv per output channel like a fused BN
(layer-sequential: mean 0 / std 1 pre-activation on synthetic road frames,
using the fp32 CPU oracle forward), then sets the head (DFL logits std 2.5,
class logits std 1.0 with a mean that yields a few hundred NMS candidates per
1080p frame and a +1 prior on the road classes 0,2,3,5,7), and writes the
per-channel weight scale and bias (scale, shift: w' = w*scale,
b' = b*scale + shift) to rvs_amd/detect/data/synthetic_calib.npz.
rvs_amd.detect.weights.synthetic_weights() reads that file as plain data.

    python tests/golden/make_yolo_scales.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conftest import road_frame  # noqa: E402
from oracle import cpu, yolo_ref  # noqa: E402

OUT = os.path.join(REPO, "road-vision-system_amd", "rvs_amd", "detect", "data",
                   "synthetic_calib.npz")
ROAD = (0, 2, 3, 5, 7)


def calibrate(variant, seed=0, H=1080, W=1920, box_std=2.5, cls_std=1.0, target_cand=0.04,
              nframes=2):
    specs, _ = yolo_ref.conv_specs(variant)
    rng = np.random.default_rng(seed)
    frames = [road_frame(H, W, seed=100 + s) for s in range(nframes)]
    geo = cpu.letterbox_geometry(H, W)
    lb = np.stack([cpu.letterbox(cpu.median(cpu.clahe_ycrcb(f), 3), geo) for f in frames])
    x = yolo_ref.preprocess(lb)
    flat = []
    for n, ci, co, k, s, act in specs:
        w = rng.normal(0, 1 / np.sqrt(ci * k * k), size=(co, ci, k, k)).astype(np.float32)
        b = rng.normal(0, 0.05, size=(co,)).astype(np.float32)
        flat += [w.ravel(), b]
    m = yolo_ref.YoloRef(variant, np.concatenate(flat))
    out = {}
    orig = yolo_ref.YoloRef.conv
    for n, ci, co, k, s, act in specs:
        stat = {}

        def conv(self, name, t, _n=n):
            w, b, st, kk, a = self.p[name]
            y = F.conv2d(t, w, b, stride=st, padding=kk // 2)
            if name == _n:
                stat["mean"] = y.mean((0, 2, 3)).numpy()
                stat["std"] = y.std((0, 2, 3)).numpy()
                raise StopIteration
            return F.silu(y) if a else y

        yolo_ref.YoloRef.conv = conv
        try:
            with torch.no_grad():
                m.forward(x)
        except StopIteration:
            pass
        yolo_ref.YoloRef.conv = orig
        t, mu = 1.0, 0.0
        if n.startswith("model.22.cv2.") and n.endswith(".2"):
            t = box_std
        is_cls = n.startswith("model.22.cv3.") and n.endswith(".2")
        if is_cls:
            t = cls_std
        sc = (t / np.maximum(stat["std"], 1e-6)).astype(np.float32)
        shift = (-stat["mean"] * sc + mu).astype(np.float32)
        if is_cls:
            shift[list(ROAD)] += 1.0
        w, b, st, kk, a = m.p[n]
        m.p[n] = (w * torch.from_numpy(sc).view(-1, 1, 1, 1), b * torch.from_numpy(sc) +
                  torch.from_numpy(shift), st, kk, a)
        out[n] = (sc, shift)
    # class logit mean: the (1 - target_cand) quantile of the per-anchor max
    # class logit lands on logit(0.25)
    with torch.no_grad():
        raw = m.forward(x).numpy()
    sig = np.clip(raw[:, 4:], 1e-7, 1 - 1e-7)
    logit = np.log(sig / (1 - sig))
    q = np.quantile(logit.max(1), 1 - target_cand)
    delta = np.float32(np.log(0.25 / 0.75) - q)
    for i in range(3):
        sc, shift = out[f"model.22.cv3.{i}.2"]
        out[f"model.22.cv3.{i}.2"] = (sc, shift + delta)
    return out


if __name__ == "__main__":
    arrays = {}
    for v, hw in ((0, (1080, 1920)), (2, (540, 960))):
        cal = calibrate(v, H=hw[0], W=hw[1])
        for n, (sc, sh) in cal.items():
            arrays[f"{v}/{n}/scale"] = sc
            arrays[f"{v}/{n}/shift"] = sh
        print("variant", v, "calibrated", len(cal), "convs")
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")
