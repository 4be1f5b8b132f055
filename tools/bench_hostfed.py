"""Host-fed frames (the PCIe-inclusive rate DESIGN.md §5 notes; never the
bench `value`): 32 x 1080p BGR frames per step in pinned host memory, copied
H2D on a copy stream while the previous step computes (double-buffered),
eager engine steps.  Prints one JSON line with the H2D-only rate, the
device-resident eager rate and the overlapped host-fed rate."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402
from bench import bench_config  # noqa: E402
from rvs_amd.engine import RoadVisionEngine  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S, H, W, K = 32, 1080, 1920, int(os.environ.get("K", 10))
dev = torch.device("cuda:0")
eng = RoadVisionEngine(bench_config(), S, (H, W), device=dev)
src = road_frames(S, 2, H, W, device=dev)
host = [src[i].cpu().pin_memory() for i in range(2)]
slots = [torch.empty_like(src[0]) for _ in range(2)]
ts = [torch.full((S,), k / 30.0, dtype=torch.float64, device=dev) for k in range(K + 3)]
copy = torch.cuda.Stream(device=dev)
for k in range(3):
    eng.step(src[k % 2], ts[k])
torch.cuda.synchronize()

t0 = time.perf_counter()
for k in range(K):
    slots[k % 2].copy_(host[k % 2], non_blocking=True)
torch.cuda.synchronize()
h2d = (time.perf_counter() - t0) / K

t0 = time.perf_counter()
for k in range(K):
    eng.step(src[k % 2], ts[k])
torch.cuda.synchronize()
dev_rate = S * K / (time.perf_counter() - t0)

done = [torch.cuda.Event(), torch.cuda.Event()]
with torch.cuda.stream(copy):
    slots[0].copy_(host[0], non_blocking=True)
    done[0].record(copy)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    cur, nxt = k % 2, (k + 1) % 2
    torch.cuda.current_stream().wait_event(done[cur])
    eng.step(slots[cur], ts[k])
    if k + 1 < K:
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(copy):
            copy.wait_event(ev)  # slot nxt was read by step k-1
            slots[nxt].copy_(host[nxt], non_blocking=True)
            done[nxt].record(copy)
torch.cuda.synchronize()
fed = S * K / (time.perf_counter() - t0)
print(json.dumps({"workload": "32 x 1080p per step, host-fed from pinned memory",
                  "h2d_ms_per_step": round(h2d * 1e3, 3),
                  "h2d_gbs": round(S * H * W * 3 / h2d / 1e9, 1),
                  "h2d_only_frames_per_s": round(S / h2d, 1),
                  "device_resident_eager_frames_per_s": round(dev_rate, 1),
                  "host_fed_overlapped_frames_per_s": round(fed, 1)}))
