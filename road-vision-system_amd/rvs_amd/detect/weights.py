"""YOLOv8 weights for the HIP detector.

The conv list (names, shapes, order) comes from the native plan in
csrc/yolo.hip (rv_yolo_conv_info) -- Ultralytics state_dict order with BN
fused.  Real checkpoints are not available in this environment
(.MISSING_LARGE_BLOBS:1 lists yolov8n.pt; there is no network), so weights are
either loaded from a local .npz / .safetensors of fused tensors keyed by the
Ultralytics module names ("model.2.m.0.cv1.weight" / ".bias"), or generated
synthetically from a seed (He-normal, calibrated so a 1080p frame yields a few
hundred NMS candidates like a trained model on a road scene).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Tuple

import numpy as np

from .. import _lib

VARIANTS = {"n": 0, "s": 1, "m": 2, "l": 3, "x": 4}
COCO80 = [
    "person", "bicycle", "car", "motorcycle", "airplane", "bus", "train", "truck", "boat",
    "traffic light", "fire hydrant", "stop sign", "parking meter", "bench", "bird", "cat", "dog",
    "horse", "sheep", "cow", "elephant", "bear", "zebra", "giraffe", "backpack", "umbrella",
    "handbag", "tie", "suitcase", "frisbee", "skis", "snowboard", "sports ball", "kite",
    "baseball bat", "baseball glove", "skateboard", "surfboard", "tennis racket", "bottle",
    "wine glass", "cup", "fork", "knife", "spoon", "bowl", "banana", "apple", "sandwich", "orange",
    "broccoli", "carrot", "hot dog", "pizza", "donut", "cake", "chair", "couch", "potted plant",
    "bed", "dining table", "toilet", "tv", "laptop", "mouse", "remote", "keyboard", "cell phone",
    "microwave", "oven", "toaster", "sink", "refrigerator", "book", "clock", "vase", "scissors",
    "teddy bear", "hair drier", "toothbrush"]


def variant_of(model_name: str) -> int:
    """'yolov8n.pt' -> 0 ... (the reference's cfg['model'], default.yaml:39)."""
    base = os.path.basename(str(model_name)).lower()
    for k, v in VARIANTS.items():
        if base.startswith(f"yolov8{k}"):
            return v
    raise ValueError(f"unsupported model '{model_name}' (YOLOv8 n/s/m/l/x only)")


def conv_list(variant: int) -> List[Tuple[str, int, int, int, int, int]]:
    """[(name, cin, cout, k, stride, silu)] in packing order."""
    lib = _lib.load()
    out = []
    info = (ctypes.c_int * 5)()
    name = ctypes.create_string_buffer(96)
    for i in range(lib.rv_yolo_num_convs(variant)):
        _lib.check(lib.rv_yolo_conv_info(variant, i, info, name, 96), "rv_yolo_conv_info")
        out.append((name.value.decode(), info[0], info[1], info[2], info[3], info[4]))
    return out


_CALIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "synthetic_calib.npz")


def synthetic_weights(variant: int, seed: int = 0) -> np.ndarray:
    """Seeded BN-fused-like weights as one flat f32 array.

    Unit-fan-in normal weights, then the per-channel scale/shift stored in
    data/synthetic_calib.npz (w' = w*scale, b' = b*scale + shift; produced
    offline by tests/golden/make_yolo_scales.py), so every conv's
    pre-activation is O(1) like a trained model's fused BN output and a road
    frame yields a few hundred NMS candidates."""
    rng = np.random.default_rng(seed)
    parts = []
    with np.load(_CALIB, allow_pickle=False) as cal:
        for name, cin, cout, k, s, act in conv_list(variant):
            w = rng.normal(0, 1 / np.sqrt(cin * k * k), size=(cout, cin, k, k)).astype(np.float32)
            b = rng.normal(0, 0.05, size=(cout,)).astype(np.float32)
            sc = cal[f"{variant}/{name}/scale"].astype(np.float32)
            sh = cal[f"{variant}/{name}/shift"].astype(np.float32)
            parts += [(w * sc[:, None, None, None]).ravel(), b * sc + sh]
    return np.concatenate(parts).astype(np.float32)


def load_weights(path: str, variant: int) -> np.ndarray:
    """Flat f32 array from a local .npz / .safetensors of fused tensors."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        tensors: Dict[str, np.ndarray] = load_file(path)
    else:
        with np.load(path, allow_pickle=False) as z:
            tensors = {k: z[k] for k in z.files}
    parts = []
    for name, cin, cout, k, s, act in conv_list(variant):
        w = np.asarray(tensors[name + ".weight"], np.float32).reshape(cout, cin, k, k)
        b = np.asarray(tensors[name + ".bias"], np.float32).reshape(cout)
        parts += [w.ravel(), b]
    return np.concatenate(parts)


def pack(variant: int, flat: np.ndarray) -> np.ndarray:
    """Device layout (bf16 [Cout16][ky][kx][Cin32] + f32 bias) as a u8 host array."""
    lib = _lib.load()
    flat = np.ascontiguousarray(flat, np.float32)
    nbytes = lib.rv_yolo_packed_bytes(variant)
    out = np.zeros(nbytes, np.uint8)
    _lib.check(lib.rv_yolo_pack(variant, flat.ctypes.data, flat.size, out.ctypes.data, nbytes),
               "rv_yolo_pack")
    return out
