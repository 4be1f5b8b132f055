"""Fingerprint of one fp8 forward (YOLOv8n 640x640, batch 1): a hash of
every activation buffer and of the raw prediction, for A/B checks of two
library builds (RV_LIB_VARIANT)."""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from conftest import road_frame  # noqa: E402
from rvs_amd.detect import weights  # noqa: E402
from rvs_amd.detect.yolo_hip import YoloEngine  # noqa: E402

dev = torch.device("cuda:0")
eng = YoloEngine(0, weights.synthetic_weights(0, seed=1), 1, (640, 640), device=dev, dtype="fp8")
lb = eng.letterbox(torch.from_numpy(road_frame(640, 640, seed=30)[None]).to(dev))
sc = eng.calibrate(lb)
raw = torch.empty((1, 84, eng.A), dtype=torch.float32, device=dev)
eng.forward_raw(lb, raw)
torch.cuda.synchronize()
ws = eng.ws.cpu().numpy()
for (name, h, w, c, es, off), s in zip(eng.buffers(1), sc):
    n = h * w * c * es
    print(f"{name:14s} {hashlib.md5(ws[off:off + n].tobytes()).hexdigest()[:12]}")
print("raw", hashlib.md5(raw.cpu().numpy().tobytes()).hexdigest()[:12],
      float(raw[:, 4:].max()))
