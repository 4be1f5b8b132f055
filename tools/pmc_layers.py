"""Per-conv-launch PMC counters of one YOLOv8n forward (B = 128, 1080p
letterbox, the bench's batch): run under rocprofv3 --pmc (one pass per
counter group, tools/gpu_pmc_layers.sh).  The autotuned configurations come
from TUNE (a tune file written by TUNE_SAVE on an unprofiled run of this
script) so the profiled run dispatches only the measured forward.  Between
marker tags 11 and 12 exactly one forward runs; LAYERS names its conv
launches in order (written to $OUT/layers.json by the unprofiled run).
  TUNE_SAVE=t.json LAYERS=l.json python tools/pmc_layers.py   (unprofiled)
  TUNE=t.json rocprofv3 --pmc ... -- python tools/pmc_layers.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from rvs_amd import _lib  # noqa: E402
from rvs_amd.detect import weights  # noqa: E402
from rvs_amd.detect.yolo_hip import YoloEngine  # noqa: E402

B = int(os.environ.get("B", 128))
V = 0
flat = weights.synthetic_weights(V)
eng = YoloEngine(V, flat, B, (1080, 1920), imgsz=640)
x = (torch.rand((B, 1080, 1920, 3), device="cuda") * 255).to(torch.uint8)
lb = eng.letterbox(x)
eng.forward_raw(lb)
lib = _lib.load()
if os.environ.get("TUNE"):
    eng.load_tuned([tuple(c) for c in json.load(open(os.environ["TUNE"]))["configs"]])
else:
    eng.autotune(lb)
    # persistent grids, as the bench runs them
    eng.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:]) for c in eng.tuned_configs()])
    if os.environ.get("TUNE_SAVE"):
        json.dump({"configs": [list(c) for c in eng.tuned_configs()]}, open(os.environ["TUNE_SAVE"], "w"))
    if os.environ.get("LAYERS"):
        lib.rv_yolo_profile_reps(eng._h, 1, 1)
        eng.forward_raw(lb)
        n = lib.rv_yolo_num_convs(V)
        ms = np.zeros(n); fl = np.zeros(n); cv = np.zeros(n, np.int32)
        lib.rv_yolo_profile_read(eng._h, ms.ctypes.data, fl.ctypes.data, cv.ctypes.data, n)
        convs = weights.conv_list(V)
        names = [convs[c][0] for c in cv if c >= 0]
        gfl = [float(f) for f, c in zip(fl, cv) if c >= 0]
        cfg = [list(c) for c, k in zip(eng.tuned_configs(), cv) if k >= 0]
        json.dump({"layers": names, "gflop": [g / 1e9 for g in gfl], "configs": cfg},
                  open(os.environ["LAYERS"], "w"))
        lib.rv_yolo_profile(eng._h, 0)
        eng.forward_raw(lb)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
_lib.call("rv_trace_marker", 11, _lib.stream_ptr())
eng.forward_raw(lb)
_lib.call("rv_trace_marker", 12, _lib.stream_ptr())
torch.cuda.synchronize()
print("pmc_layers done")
