"""Where conv_patch_kernel's wave time goes (timing build -DRV_PHASE_PROF,
librvhip_phase.so: tools/build_defs_variant.sh NAME=phase DEFS=-DRV_PHASE_PROF):
s_memtime cycles per phase summed over every wave of the B = 128 forward's
patch launches -- prologue, next-step DMA issue, compute, epilogue,
end-of-step barrier (incl. the vmcnt wait for the next stage).
  RV_LIB_VARIANT=phase python tools/conv_phase.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import torch  # noqa: E402
from rvs_amd import _lib  # noqa: E402
from rvs_amd.detect import weights  # noqa: E402
from rvs_amd.detect.yolo_hip import YoloEngine  # noqa: E402

B = int(os.environ.get("B", 128))
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
eng = YoloEngine(0, weights.synthetic_weights(0), B, (H, W), imgsz=640)
x = (torch.rand((B, H, W, 3), device="cuda") * 255).to(torch.uint8)
lb = eng.letterbox(x)
eng.forward_raw(lb)
eng.autotune(lb)
if not os.environ.get("KEEP_PERSIST"):  # B=1: keep the tuned grids
    eng.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:]) for c in eng.tuned_configs()])
lib = _lib.load()
f = lib.rv_conv_phase_read
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
eng.forward_raw(lb)
torch.cuda.synchronize()
f(buf, 1)
N = 3
for _ in range(N):
    eng.forward_raw(lb)
    torch.cuda.synchronize()
f(buf, 0)
v = list(buf)
names = ["prologue", "dma issue", "compute", "epilogue", "barrier+wait"]
tot = sum(v[:5])
print(f"{N} forwards: {v[6] // N} waves and {v[5] // N} wave-steps per forward; "
      f"{tot / max(v[6], 1):.0f} cycles per wave")
for i, n in enumerate(names):
    print(f"  {n:14s} {v[i] / tot:6.3f}  {v[i] / max(v[5], 1):8.0f} cycles per wave-step")
