"""Per-conv device time of the YOLOv8 forward (HIP events, rv_yolo_profile)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from rvs_amd import _lib
from rvs_amd.detect import weights
from rvs_amd.detect.yolo_hip import YoloEngine

B = int(os.environ.get("B", 32))
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
V = int(os.environ.get("V", 0))
N = int(os.environ.get("N", 10))
DT = os.environ.get("DTYPE", "bf16")
flat = weights.synthetic_weights(V)
eng = YoloEngine(V, flat, B, (H, W), imgsz=int(os.environ.get("IMGSZ", 640)), dtype=DT)
x = (torch.rand((B, H, W, 3), device="cuda") * 255).to(torch.uint8)
lb = eng.letterbox(x)
if DT == "fp8":
    eng.calibrate(lb)
for _ in range(3):
    eng.forward_raw(lb)
if not os.environ.get("NO_TUNE"):
    eng.autotune(lb)
lib = _lib.load()
REPS = int(os.environ.get("REPS", 5))  # launches per event pair (event overhead)
lib.rv_yolo_profile_reps(eng._h, N, REPS)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
for _ in range(N):
    eng.forward_raw(lb)
e.record()
torch.cuda.synchronize()
fwd = s.elapsed_time(e) / N
n = lib.rv_yolo_num_convs(V)
ms = np.zeros(n); fl = np.zeros(n); cv = np.zeros(n, np.int32)
nf = lib.rv_yolo_profile_read(eng._h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, n)
convs = weights.conv_list(V)
tot = 0
rows = []
cfgs = eng.tuned_configs()
for i in range(n):
    if cv[i] < 0:
        continue
    name, ci, co, k, st, act = convs[cv[i]]
    t = ms[i] / nf
    tot += t
    rows.append((t, name, ci, co, k, st, fl[i], cfgs[i] if i < len(cfgs) else ()))
print(f"{DT} B={B} {H}x{W} forward {fwd:.3f} ms (events), conv sum {tot:.3f} ms over {len(rows)} launches")
for t, name, ci, co, k, st, f, c in (rows if os.environ.get("ORDER") else sorted(rows, reverse=True)[:40]):
    print(f"{t*1e3:8.1f} us {f/1e9:7.2f} GF {f/t/1e9:7.1f} TF/s  {name:22s} {ci:4d}->{co:4d} k{k} s{st}  cfg {c}")
