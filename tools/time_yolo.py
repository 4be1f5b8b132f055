"""Device timing of the detector stages at 1080p (HIP events)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from conftest import road_frame
from rvs_amd.detect import weights
from rvs_amd.detect.yolo_hip import YoloEngine

B = int(os.environ.get("B", 32))
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
flat = weights.synthetic_weights(0)
eng = YoloEngine(0, flat, B, (H, W), classes_keep=[0, 2, 3, 5, 7])
fr = np.stack([road_frame(H, W, seed=s) for s in range(4)])
x = torch.from_numpy(fr).cuda().repeat(B // 4, 1, 1, 1).contiguous()
lb = eng.letterbox(x)


def t(fn, n=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


ms_f = t(lambda: eng.forward_raw(lb))
ms_n = t(lambda: eng.nms(B))
ms_all = t(lambda: eng.run(x))
flops = 2 * 2.623e9 * B if (H, W) == (1080, 1920) else 2 * 4.371e9 * B
print(f"B={B} forward {ms_f:.3f} ms ({flops / ms_f / 1e9:.1f} TFLOP/s)  nms {ms_n:.3f} ms  "
      f"letterbox+fwd+nms {ms_all:.3f} ms -> {B / ms_all * 1e3:.0f} fps")
print("cand per image", eng.cand_n[:B].cpu().numpy()[:8], "dets", eng.det_n[:B].cpu().numpy()[:8])
