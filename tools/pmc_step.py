"""Two eager bench steps (32 streams x 1080p, full chain) for rocprofv3
--pmc passes: every dispatch of the second step is one row per counter in
counter_collection.csv (tools/pmc_report.py summarises it)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.engine import LanedEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
dev = torch.device("cuda:0")
eng = LanedEngine(bench.bench_config(), S, (1080, 1920), device=dev, lanes=1)
frames = road_frames(S, 2, 1080, 1920, device=dev)
ts = torch.tensor([[f / 30.0] * S for f in range(2)], dtype=torch.float64, device=dev)
for f in range(2):
    eng.step(frames[f], ts[f])
torch.cuda.synchronize()
print("pmc_step done")
