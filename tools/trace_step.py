"""Replay the bench step (autotuned convs, OverlappedSteps graphs) for a
kernel-trace timeline: 2 eager warmup steps, autotune, then N steps.  Used
under `rocprofv3 --kernel-trace --output-format csv`; analyse with
tools/layer_table.py / tools/timeline.py."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.engine import OverlappedSteps, RoadVisionEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
N = int(os.environ.get("N", 20))
dev = torch.device("cuda:0")
eng = RoadVisionEngine(bench.bench_config(), S, (1080, 1920), device=dev)
frames = road_frames(S, 2 + N, 1080, 1920, device=dev)
ts = torch.tensor([[f / 30.0] * S for f in range(2 + N)], dtype=torch.float64, device=dev)
for f in range(2):
    eng.step(frames[f], ts[f])
if not os.environ.get("NO_TUNE"):
    eng.autotune(frames[0])
torch.cuda.synchronize()
run = OverlappedSteps(eng, [frames[2 + k] for k in range(N)], [ts[2 + k] for k in range(N)],
                      depth=int(os.environ.get("RV_PIPE_DEPTH", 3)))
torch.cuda.synchronize()
time.sleep(0.05)
t = time.perf_counter()
run.run()
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t) / N * 1e3:.3f} ms/step over {N} steps")
