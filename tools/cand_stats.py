"""Candidates per image (anchors with best class score > conf) that reach NMS
on the bench workload (synthetic road frames, synthetic LSUV weights)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch
from bench import H, W, bench_config
from rvs_amd.engine import RoadVisionEngine
from rvs_amd.synth import road_frames

S = int(os.environ.get("S", 32))
eng = RoadVisionEngine(bench_config(), S, (H, W), device="cuda")
fr = road_frames(S, 3, H, W, device="cuda")
ts = torch.zeros(S, dtype=torch.float64, device="cuda")
for f in range(3):
    out = eng.step(fr[f], ts + f / 30)
torch.cuda.synchronize()
n = eng.detector.cand_n[:S].cpu()  # written by the NMS
print("fused_letterbox", eng.fused_letterbox)
print("candidates/image min %d median %d max %d" % (n.min(), n.median(), n.max()))
print("detections/image", out["det_n"].cpu().tolist())
