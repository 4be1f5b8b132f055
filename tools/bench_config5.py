"""BASELINE config 5 timing: fog/rain frames made on device -> YOLOv8m at
1280x1280 -> NMS, batch 16, one MI355X (bf16; the fp8 variant is not built).

Prints one JSON line: per-stage device times (HIP events on the launch
stream), frames/s of fog+detector, the fog kernel's HBM GB/s (6 B/pixel
algorithmic: 3 B read + 3 B written) and the forward's TFLOP/s
(315.7 GFLOP/frame).  AUTOTUNE=1 runs the per-layer conv
autotuner first (bit-identical configs only).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from conftest import road_frame  # noqa: E402
from rvs_amd.augment import FogSynthesizer  # noqa: E402
from rvs_amd.detect import weights  # noqa: E402
from rvs_amd.detect.yolo_hip import YoloEngine  # noqa: E402

B, H, W = int(os.environ.get("B", 16)), 1280, 1280
dev = torch.device("cuda:0")
clean = torch.from_numpy(np.stack([road_frame(H, W, seed=70 + b) for b in range(4)]))
clean = clean.to(dev).repeat(B // 4, 1, 1, 1).contiguous()
syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=dev)
draws = [syn.draw(H, W) for _ in range(B)]
prep = syn.prepare(draws)
fog = syn.synthesize_batch(clean, prepared=prep)
eng = YoloEngine(2, weights.synthetic_weights(2, seed=0), B, (H, W), imgsz=1280, device=dev,
                 classes_keep=[0, 2, 3, 5, 7])
lb = eng.letterbox(fog)
if os.environ.get("AUTOTUNE", "0") == "1":
    eng.autotune(lb, reps=2)


def t(fn, n=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


ms_fog = t(lambda: syn.synthesize_batch(clean, out=fog, prepared=prep))
ms_fwd = t(lambda: eng.forward_raw(lb))
ms_nms = t(lambda: eng.nms(B))
ms_all = t(lambda: (syn.synthesize_batch(clean, out=fog, prepared=prep), eng.run(fog)))
gflop = 315.7 * B
print(json.dumps({
    "workload": "config 5: fog/rain 1280x1280 -> YOLOv8m imgsz 1280 -> NMS, batch %d" % B,
    "dtype": "bf16", "autotune": os.environ.get("AUTOTUNE", "0") == "1",
    "ms_fog": round(ms_fog, 4), "ms_forward": round(ms_fwd, 4), "ms_nms": round(ms_nms, 4),
    "ms_step": round(ms_all, 4), "frames_per_s": round(B / ms_all * 1e3, 1),
    "fog_hbm_gbs": round(6 * H * W * B / ms_fog / 1e6, 1),
    "forward_tflops": round(gflop / ms_fwd, 1),
    "forward_mfma_frac": round(gflop / ms_fwd / 2500.0, 4),
    "dets_per_frame": eng.det_n[:B].float().mean().item()}))
