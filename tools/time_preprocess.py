"""Quick device timing of the preprocess kernels (HIP events)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from conftest import road_frame
from rvs_amd import kernels

B, H, W = int(os.environ.get("B", 32)), 1080, 1920
frames = np.stack([road_frame(H, W, seed=s) for s in range(4)])
x = torch.from_numpy(frames).cuda().repeat(B // 4, 1, 1, 1).contiguous()
out = torch.empty_like(x)
ws = torch.empty(kernels.clahe_ws_bytes(B, 8), dtype=torch.uint8, device="cuda")
geo = kernels.letterbox_geometry(H, W)
lb = torch.empty((B, geo[0], geo[1], 3), dtype=torch.uint8, device="cuda")


def t(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


frame_bytes = H * W * 3
for name, fn, nbytes in [
    ("clahe_ycrcb", lambda: kernels.clahe_ycrcb(x, 8, 2.0, out=out, ws=ws), 3 * frame_bytes),
    ("median3", lambda: kernels.median(x, 3, out=out), 2 * frame_bytes),
    ("clahe_median", lambda: kernels.clahe_median(x, 8, 2.0, 3, out=out, ws=ws), 3 * frame_bytes),
    ("clahe_med_lb", lambda: kernels.clahe_median_letterbox(x, 8, 2.0, 3, geo, out=out, lb_out=lb,
                                                             ws=ws), 3 * frame_bytes),
    ("letterbox", lambda: kernels.letterbox(out, geo, out=lb), frame_bytes / 3 + lb[0].numel()),
]:
    ms = t(fn)
    print(f"{name:14s} B={B} {ms:8.3f} ms  {B / ms * 1e3:10.0f} fps  "
          f"{B * nbytes / ms / 1e6:8.1f} GB/s (algorithmic)")
