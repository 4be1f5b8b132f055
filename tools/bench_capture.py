"""Capture-fed frames through the whole front end (§8(f)4; a PCIe-inclusive
rate, never the bench `value`): S camera streams, each a YUV4MPEG2 file of F
1080p frames (looped), read by the native reader threads into pinned slots,
uploaded as NV12 by MultiStreamCapture on its copy stream one batch ahead,
converted to BGR on the device, then one RoadVisionEngine step per batch
(eager launches) with the result hand-back.  Prints one JSON line: frames/s
of the capture-fed loop, the capture alone (no engine), and the
device-resident eager rate on the same engine for reference."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import bench_config  # noqa: E402
from rvs_amd.engine import RoadVisionEngine  # noqa: E402
from rvs_amd.io_video import MultiStreamCapture, write_y4m  # noqa: E402
from rvs_amd.synth import road_frames  # noqa: E402

S = int(os.environ.get("S", 32))
F = int(os.environ.get("F", 4))
K = int(os.environ.get("K", 30))
H, W = 1080, 1920


def main():
    dev = torch.device("cuda:0")
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    frames = road_frames(S, F, H, W, device=dev).cpu().numpy()
    paths = []
    t0 = time.perf_counter()
    for s in range(S):
        p = os.path.join(tmp, f"cam{s}.y4m")
        write_y4m(p, [frames[f, s] for f in range(F)])
        paths.append(p)
    gen_s = time.perf_counter() - t0
    eng = RoadVisionEngine(bench_config(), S, (H, W), device=dev)
    # capture alone
    cap = MultiStreamCapture(paths, device=dev, loop=True, nbuf=4)
    for _ in range(3):
        cap.next_batch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        cap.next_batch()
    torch.cuda.synchronize()
    cap_only = S * K / (time.perf_counter() - t0)
    # capture-fed engine steps
    for k in range(3):
        fr, ts, _ = cap.next_batch()
        eng.step(fr, ts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        fr, ts, _ = cap.next_batch()
        eng.step(fr, ts)
    torch.cuda.synchronize()
    fed = S * K / (time.perf_counter() - t0)
    pinned = cap.pinned
    cap.close()
    # device-resident eager steps on the same engine
    src = road_frames(S, 2, H, W, device=dev)
    tsd = torch.zeros(S, dtype=torch.float64, device=dev)
    for k in range(3):
        eng.step(src[k % 2], tsd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        eng.step(src[k % 2], tsd)
    torch.cuda.synchronize()
    resident = S * K / (time.perf_counter() - t0)
    eng.close()
    for p in paths:
        os.remove(p)
    print(json.dumps({
        "metric": "capture-fed frames/s @1080p (y4m files -> reader threads -> pinned NV12 -> "
                  "H2D -> device NV12->BGR -> full chain, eager steps)",
        "value": round(fed, 1), "unit": "frames/s", "streams": S, "steps": K,
        "capture_only_fps": round(cap_only, 1), "device_resident_eager_fps": round(resident, 1),
        "pinned_slots": bool(pinned), "nv12_bytes_per_frame": H * W * 3 // 2,
        "h2d_gbs_at_capture_rate": round(cap_only * H * W * 1.5 / 1e9, 2),
        "y4m_generation_s": round(gen_s, 1)}))


if __name__ == "__main__":
    main()
