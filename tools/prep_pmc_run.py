"""Three launches of the fused preprocess chain (CLAHE LUT + med3 +
letterbox) on 32 synthetic 1080p frames, for rocprofv3 --pmc passes
(tools/gpu_pmc_prep.sh); counters are per family totals / launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from conftest import road_frame  # noqa: E402
from rvs_amd import kernels  # noqa: E402

B, H, W = 32, 1080, 1920
frames = np.stack([road_frame(H, W, seed=s) for s in range(4)])
x = torch.from_numpy(frames).cuda().repeat(B // 4, 1, 1, 1).contiguous()
out = torch.empty_like(x)
ws = torch.empty(kernels.clahe_ws_bytes(B, 8), dtype=torch.uint8, device="cuda")
geo = kernels.letterbox_geometry(H, W)
lb = torch.empty((B, geo[0], geo[1], 3), dtype=torch.uint8, device="cuda")
for _ in range(int(os.environ.get("REPS", 3))):
    kernels.clahe_median_letterbox(x, 8, 2.0, 3, geo, out=out, lb_out=lb, ws=ws)
torch.cuda.synchronize()
print("done", flush=True)
