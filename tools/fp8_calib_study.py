"""fp8 conditioning of the synthetic YOLOv8m weights (offline study, CPU).

For a smooth fraction `smooth` of the base weights (rvs_amd.detect.weights.
base_weights) the weights are calibrated like tests/golden/make_yolo_scales.py
does (per-channel pre-activation std / mean, head logits), then on synthetic
road frames at 640x640 (the fp8 parity test's geometry) this measures:
  * the fp8 oracle (YoloRef quant="fp8", its own per-buffer scales) against
    itself with every activation perturbed by a relative N(0, eps) before its
    fp8 rounding (what the GPU's inexact fp8 MFMA accumulation does:
    tools/fp8_probe.hip, |err| up to 2^-11.8 of the |product| sum): the share
    of detections kept (same class, IoU >= 0.9) -- the floor a GPU-vs-oracle
    test can ask for;
  * fp8 against fp32 (IoU 0.9 and 0.5), and the detections per frame.
usage: python tools/fp8_calib_study.py SMOOTH [SMOOTH ...]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import road_frame  # noqa: E402
from oracle import cpu, yolo_ref as Y  # noqa: E402
import make_yolo_scales as mys  # noqa: E402
from rvs_amd.detect.weights import base_weights  # noqa: E402

KEEP = [0, 2, 3, 5, 7]


def flat_for(variant, cal, smooth, seed=0):
    rng = np.random.default_rng(seed)
    parts = []
    for i, (n, ci, co, k, s, act) in enumerate(Y.conv_specs(variant)[0]):
        w, b = base_weights(rng, seed, i, ci, co, k, smooth)
        sc, sh = cal[n]
        parts += [(w * sc[:, None, None, None]).ravel(), b * sc + sh]
    return np.concatenate(parts).astype(np.float32)


class Perturbed(Y.YoloRef):
    eps = 0.0

    def Q(self, t, buf):
        if self.quant == "fp8" and self.amax is None and self.eps > 0:
            t = t * (1 + self.eps * torch.randn_like(t))
        return super().Q(t, buf)


def match(a, b, iou=0.9):
    tot = hit = 0
    for x, y in zip(a, b):
        for r in x:
            tot += 1
            if len(y) == 0:
                continue
            x1 = np.maximum(y[:, 0], r[0]); y1 = np.maximum(y[:, 1], r[1])
            x2 = np.minimum(y[:, 2], r[2]); y2 = np.minimum(y[:, 3], r[3])
            inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
            u = (y[:, 2] - y[:, 0]) * (y[:, 3] - y[:, 1]) + (r[2] - r[0]) * (r[3] - r[1]) - inter
            hit += bool(((inter / np.maximum(u, 1e-9) >= iou) & (y[:, 5] == r[5])).any())
    return hit, tot


def study(smooth, variant=2, H=640, W=640, eps=3e-4, nframes=2):
    t0 = time.time()
    box_std = float(os.environ.get("BOX_STD", "0.7"))
    cal = mys.calibrate(variant, H=540, W=960, mu=mys.MU, box_std=box_std, target_cand=0.012,
                        road_prior=3.0, smooth=smooth)
    flat = flat_for(variant, cal, smooth)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=20 + b)), 3)
                   for b in range(nframes)])
    geo = cpu.letterbox_geometry(H, W)
    x = Y.preprocess(np.stack([cpu.letterbox(f, geo) for f in fr]))
    sc = Y.fp8_calibration(variant, flat, x)
    hw = (geo[0], geo[1])
    post = lambda raw: Y.postprocess(raw, hw, (H, W), classes_keep=KEEP)  # noqa: E731
    d8 = post(Y.YoloRef(variant, flat, quant="fp8", scales=sc).forward(x).numpy())
    m = Perturbed(variant, flat, quant="fp8", scales=sc)
    m.eps = eps
    torch.manual_seed(1)
    dp = post(m.forward(x).numpy())
    d32 = post(Y.YoloRef(variant, flat).forward(x).numpy())
    a, b = match(d8, dp), match(dp, d8)
    c, d = match(d32, d8), match(d8, d32)
    e, f = match(d32, d8, 0.5), match(d8, d32, 0.5)
    print(f"smooth {smooth} box_std {box_std}: dets/frame {[len(v) for v in d8]} fp32 {[len(v) for v in d32]}; "
          f"fp8 vs perturbed fp8 (eps {eps}) IoU0.9 {a[0]}/{a[1]} {b[0]}/{b[1]}; "
          f"fp8 vs fp32 IoU0.9 {c[0]}/{c[1]} {d[0]}/{d[1]}, IoU0.5 {e[0]}/{e[1]} {f[0]}/{f[1]} "
          f"({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    import rvs_amd.detect.weights as wts
    wts.SMOOTH_KERNEL = os.environ.get("KERNEL", "delta")
    torch.set_num_threads(int(os.environ.get("THREADS", "8")))
    for s in sys.argv[1:]:
        study(float(s), eps=float(os.environ.get("EPS", "3e-4")), nframes=int(os.environ.get("NF", "2")))
