"""Replay the bench step (HIP graphs, RV_LANES lanes) for a kernel-trace
timeline: 2 eager warmup steps, then N graph replays.  Used under
`rocprofv3 --kernel-trace --output-format csv`; analyse with tools/timeline.py."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rvs_amd.engine import LanedEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
N = int(os.environ.get("N", 20))
L = int(os.environ.get("RV_LANES", 1))
dev = torch.device("cuda:0")
cfg = bench.bench_config()
eng = LanedEngine(cfg, S, (1080, 1920), device=dev, lanes=L)
frames = road_frames(S, 2 + N, 1080, 1920, device=dev)
ts = torch.tensor([[f / 30.0] * S for f in range(2 + N)], dtype=torch.float64, device=dev)
for f in range(2):
    eng.step(frames[f], ts[f])
torch.cuda.synchronize()
graphs = [eng.capture(frames[2 + k], ts[2 + k])[0] for k in range(N)]
torch.cuda.synchronize()
time.sleep(0.05)
t = time.perf_counter()
for g in graphs:
    g.replay()
torch.cuda.synchronize()
print(f"lanes {L}: {(time.perf_counter() - t) / N * 1e3:.3f} ms/step over {N} replays")
