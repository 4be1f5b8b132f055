"""Host-fed frames (the PCIe-inclusive rate DESIGN.md §5 notes; never the
bench `value`): 32 x 1080p frames per step in pinned host memory, copied
H2D on a copy stream while the previous step computes (double-buffered),
eager engine steps.  Two host formats: BGR (3 B/pixel, what the reference's
capture hands over) and NV12 (1.5 B/pixel, what a hardware decoder hands
over; converted on device by rv_nv12_to_bgr_u8 before the step).  Prints one
JSON line with the H2D-only rates, the device-resident eager rate and the
overlapped host-fed rates."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402
from bench import bench_config  # noqa: E402
from rvs_amd import kernels  # noqa: E402
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

# NV12 host frames (random planes: the conversion cost does not depend on
# content), converted on device into the BGR slot the step reads
nv_host = [torch.randint(0, 256, (S, H * 3 // 2, W), dtype=torch.uint8).pin_memory()
           for _ in range(2)]
nv_dev = [torch.empty((S, H * 3 // 2, W), dtype=torch.uint8, device=dev) for _ in range(2)]
t0 = time.perf_counter()
for k in range(K):
    nv_dev[k % 2].copy_(nv_host[k % 2], non_blocking=True)
torch.cuda.synchronize()
h2d_nv = (time.perf_counter() - t0) / K
s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s0.record()
for k in range(K):
    kernels.nv12_to_bgr(nv_dev[k % 2], out=slots[k % 2])
s1.record()
torch.cuda.synchronize()
conv_ms = s0.elapsed_time(s1) / K
with torch.cuda.stream(copy):
    nv_dev[0].copy_(nv_host[0], non_blocking=True)
    done[0].record(copy)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    cur, nxt = k % 2, (k + 1) % 2
    torch.cuda.current_stream().wait_event(done[cur])
    kernels.nv12_to_bgr(nv_dev[cur], out=slots[cur])
    eng.step(slots[cur], ts[k])
    if k + 1 < K:
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(copy):
            copy.wait_event(ev)
            nv_dev[nxt].copy_(nv_host[nxt], non_blocking=True)
            done[nxt].record(copy)
torch.cuda.synchronize()
fed_nv = S * K / (time.perf_counter() - t0)
print(json.dumps({"workload": "32 x 1080p per step, host-fed from pinned memory",
                  "h2d_ms_per_step": round(h2d * 1e3, 3),
                  "h2d_gbs": round(S * H * W * 3 / h2d / 1e9, 1),
                  "h2d_only_frames_per_s": round(S / h2d, 1),
                  "device_resident_eager_frames_per_s": round(dev_rate, 1),
                  "host_fed_overlapped_frames_per_s": round(fed, 1),
                  "nv12_h2d_ms_per_step": round(h2d_nv * 1e3, 3),
                  "nv12_h2d_only_frames_per_s": round(S / h2d_nv, 1),
                  "nv12_to_bgr_ms_per_step": round(conv_ms, 4),
                  "nv12_to_bgr_hbm_gbs": round(S * H * W * 4.5 / (conv_ms * 1e-3) / 1e9, 1),
                  "host_fed_nv12_overlapped_frames_per_s": round(fed_nv, 1)}))
