"""Two eager bench steps (autotuned convs) (32 streams x 1080p, full chain) for rocprofv3
--pmc passes: every dispatch of the second step is one row per counter in
counter_collection.csv (tools/pmc_report.py summarises it)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.engine import RoadVisionEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
dev = torch.device("cuda:0")
eng = RoadVisionEngine(bench.bench_config(), S, (1080, 1920), device=dev)
frames = road_frames(S, 2, 1080, 1920, device=dev)
ts = torch.tensor([[f / 30.0] * S for f in range(2)], dtype=torch.float64, device=dev)
eng.step(frames[0], ts[0])
eng.autotune(frames[0])  # the bench's kernel configurations
eng.step(frames[1], ts[1])
torch.cuda.synchronize()
print("pmc_step done")
