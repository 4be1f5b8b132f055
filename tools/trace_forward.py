"""Run the batched YOLOv8 forward N times (no HIP-event profiling) so that a
rocprofv3 --kernel-trace of this process gives clean per-launch durations."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch
from rvs_amd.detect import weights
from rvs_amd.detect.yolo_hip import YoloEngine

B = int(os.environ.get("B", 32))
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
V = int(os.environ.get("V", 0))
N = int(os.environ.get("N", 10))
eng = YoloEngine(V, weights.synthetic_weights(V), B, (H, W))
x = (torch.rand((B, H, W, 3), device="cuda") * 255).to(torch.uint8)
lb = eng.letterbox(x)
for _ in range(3):
    eng.forward_raw(lb)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(N):
    eng.forward_raw(lb)
e.record()
torch.cuda.synchronize()
print(f"B={B} {H}x{W} forward {s.elapsed_time(e) / N:.3f} ms")
