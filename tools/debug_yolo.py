"""Diagnostic: GPU raw vs quantised oracle, error by level / location."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from conftest import road_frame
from oracle import cpu, yolo_ref
from rvs_amd.detect import weights
from rvs_amd.detect.yolo_hip import YoloEngine

H, W = int(os.environ.get("H", 640)), int(os.environ.get("W", 640))
flat = weights.synthetic_weights(0)
eng = YoloEngine(0, flat, 1, (H, W))
fr = cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=0)), 3)[None]
lb = eng.letterbox(torch.from_numpy(fr).cuda())
raw = torch.empty((1, 84, eng.A), dtype=torch.float32, device="cuda")
eng.forward_raw(lb, raw, candidates=False)
got = raw.cpu().numpy()[0]
for q in (True, False):
    ref = yolo_ref.YoloRef(0, flat, quant=q).forward(yolo_ref.preprocess(lb.cpu().numpy())).numpy()[0]
    db = np.abs(got[:4] - ref[:4]).max(0)
    ds = np.abs(got[4:] - ref[4:]).max(0)
    hs = [eng.in_h // s * (eng.in_w // s) for s in (8, 16, 32)]
    st = np.cumsum([0] + hs)
    for l in range(3):
        seg = slice(st[l], st[l + 1])
        w = eng.in_w // (8 << l)
        bad = np.where(db[seg] > 2)[0]
        print(f"quant={q} level {l}: box max {db[seg].max():.2f} p99 {np.percentile(db[seg], 99):.3f} "
              f"bad {len(bad)} score max {ds[seg].max():.4f}; bad yx {[(int(i // w), int(i % w)) for i in bad[:12]]}")
