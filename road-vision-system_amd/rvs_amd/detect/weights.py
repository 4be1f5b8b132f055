"""YOLOv8 weights for the HIP detector.

The conv list (names, shapes, order) comes from the native plan in
csrc/yolo.hip (rv_yolo_conv_info) -- Ultralytics state_dict order with BN
fused.  Real checkpoints are not available in this environment
(.MISSING_LARGE_BLOBS:1 lists yolov8n.pt; there is no network), so weights are
either loaded from a local Ultralytics state_dict (load_weights: .safetensors,
.npz, or a tensors-only torch file read with weights_only=True -- never a
pickle), or generated synthetically from a seed.

load_weights accepts the Ultralytics DetectionModel state_dict keys as they
are before and after ``model.fuse()`` (the reference calls it,
src/detect/yolo_ultralytics.py:16-17):
  * unfused Conv blocks: ``model.N[...].conv.weight`` + ``.bn.weight / .bn.bias
    / .bn.running_mean / .bn.running_var`` -- folded here exactly as
    ultralytics.utils.torch_utils.fuse_conv_and_bn does (BatchNorm2d eps =
    1e-3, set by initialize_weights), in float32;
  * fused Conv blocks: ``model.N[...].conv.weight`` + ``.conv.bias``;
  * the Detect head's plain 1x1 convs: ``model.22.cv2.i.2.weight / .bias``;
  * the plan's own names (``model.2.m.0.cv1.weight / .bias``, round-1 files).
The DFL conv (``model.22.dfl.conv.weight``, a fixed arange) and
``num_batches_tracked`` are ignored.
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


SMOOTH_KERNEL = "delta"  # spatial profile of the coherent part: "delta" (centre tap) or "blur"


def base_weights(rng, seed: int, idx: int, cin: int, cout: int, k: int, smooth: float):
    """Base (pre-calibration) weights and bias of conv `idx`: unit-fan-in
    He-normal weights (drawn from `rng`, the same stream for every `smooth`),
    mixed with weight `smooth` in [0, 1) of a channel-coherent part -- per
    output channel a signed gain times one positive per-input-channel profile
    on the centre tap (SMOOTH_KERNEL), rows scaled to the same norm as the
    random part.  Trained conv filters are spatially smooth and
    their inputs redundant, so noise added to an activation (quantisation,
    accumulation order) is averaged down layer by layer; pure random weights
    pass it on at full strength (the chaotic regime)."""
    w = rng.normal(0, 1 / np.sqrt(cin * k * k), size=(cout, cin, k, k)).astype(np.float32)
    b = rng.normal(0, 0.05, size=(cout,)).astype(np.float32)
    if smooth > 0:
        srng = np.random.default_rng([seed, 7919, idx])
        g = np.zeros((k, k))
        if SMOOTH_KERNEL == "blur" and k == 3:
            g1 = np.array([1.0, 2.0, 1.0])
            g = np.outer(g1, g1)
        else:
            g[k // 2, k // 2] = 1.0
        u = srng.uniform(0.5, 1.5, cin)
        a = srng.choice([-1.0, 1.0], cout) * srng.uniform(0.5, 1.5, cout)
        st = a[:, None, None, None] * u[None, :, None, None] * g[None, None]
        st /= np.sqrt((st ** 2).sum(axis=(1, 2, 3), keepdims=True))
        w = (np.sqrt(1 - smooth) * w + np.sqrt(smooth) * st).astype(np.float32)
    return w, b


def synthetic_weights(variant: int, seed: int = 0) -> np.ndarray:
    """Seeded BN-fused-like weights as one flat f32 array.

    Base weights (base_weights: He-normal, for some variants mixed with a
    smooth part, data/synthetic_calib.npz "<variant>/smooth"), then the
    per-channel scale/shift stored in data/synthetic_calib.npz (w' =
    w*scale, b' = b*scale + shift; produced offline by
    tests/golden/make_yolo_scales.py), so every conv's pre-activation is O(1)
    like a trained model's fused BN output and a road frame yields a few
    hundred NMS candidates."""
    rng = np.random.default_rng(seed)
    parts = []
    with np.load(_CALIB, allow_pickle=False) as cal:
        smooth = float(cal[f"{variant}/smooth"]) if f"{variant}/smooth" in cal.files else 0.0
        for i, (name, cin, cout, k, s, act) in enumerate(conv_list(variant)):
            w, b = base_weights(rng, seed, i, cin, cout, k, smooth)
            sc = cal[f"{variant}/{name}/scale"].astype(np.float32)
            sh = cal[f"{variant}/{name}/shift"].astype(np.float32)
            parts += [(w * sc[:, None, None, None]).ravel(), b * sc + sh]
    return np.concatenate(parts).astype(np.float32)


BN_EPS = 1e-3  # ultralytics.nn.tasks.initialize_weights: BatchNorm2d.eps = 1e-3


def fold_bn(w: np.ndarray, gamma: np.ndarray, beta: np.ndarray, mean: np.ndarray,
            var: np.ndarray, bias=None, eps: float = BN_EPS):
    """ultralytics.utils.torch_utils.fuse_conv_and_bn in float32 torch ops:
    w_bn = diag(gamma / sqrt(eps + var)); W = w_bn @ w; b = w_bn @ b_conv +
    (beta - gamma * mean / sqrt(var + eps)).  torch's own sqrt / div / mul
    are used (torch's CPU sqrt is not always the correctly rounded one, and
    the reference folds with it); the diagonal matmuls are evaluated as the
    exact per-row products they denote (a BLAS sgemm of a diagonal matrix
    returns some of them 1 ulp off, platform-dependently)."""
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32))  # noqa: E731
    w, gamma, beta, mean, var = t(w), t(gamma), t(beta), t(mean), t(var)
    scale = gamma.div(torch.sqrt(eps + var))
    wf = scale.view(-1, *([1] * (w.dim() - 1))) * w
    b_conv = torch.zeros_like(beta) if bias is None else t(bias)
    b_bn = beta - gamma.mul(mean).div(torch.sqrt(var + eps))
    return wf.numpy(), (scale * b_conv + b_bn).numpy()


def read_state_dict(path: str) -> Dict[str, np.ndarray]:
    """Tensors of a local checkpoint, with loaders that execute nothing
    from the file: .safetensors, .npz (allow_pickle=False), or a torch file
    of plain tensors (torch.load(weights_only=True))."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        return dict(load_file(path))
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: expected a state_dict of tensors (save model.state_dict())")
    return {k: v.detach().float().numpy() if hasattr(v, "detach") else np.asarray(v)
            for k, v in sd.items()}


def _strip_prefix(t: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    # YOLO(...).state_dict() nests the DetectionModel under "model."
    if any(k.startswith("model.model.") for k in t):
        t = {k[len("model."):]: v for k, v in t.items() if k.startswith("model.")}
    return t


def flat_from_state_dict(tensors: Dict[str, np.ndarray], variant: int) -> np.ndarray:
    """Flat f32 weights (the plan's conv order) from an Ultralytics
    DetectionModel state_dict, fused or not (see the module docstring)."""
    t = _strip_prefix(tensors)
    parts = []
    for name, cin, cout, k, s, act in conv_list(variant):
        shape = (cout, cin, k, k)
        if name + ".conv.weight" in t:  # Conv block (conv + bn + SiLU)
            w = np.asarray(t[name + ".conv.weight"], np.float32).reshape(shape)
            if name + ".bn.running_var" in t:
                w, b = fold_bn(w, t[name + ".bn.weight"], t[name + ".bn.bias"],
                               t[name + ".bn.running_mean"], t[name + ".bn.running_var"],
                               t.get(name + ".conv.bias"))
            elif name + ".conv.bias" in t:
                b = np.asarray(t[name + ".conv.bias"], np.float32)
            else:
                raise KeyError(f"{name}: neither .bn.* nor .conv.bias in the state_dict")
        elif name + ".weight" in t:  # Detect's plain nn.Conv2d / the plan's own names
            w = np.asarray(t[name + ".weight"], np.float32).reshape(shape)
            b = np.asarray(t[name + ".bias"], np.float32)
        else:
            raise KeyError(f"{name}: no weights in the state_dict "
                           f"(expected {name}.conv.weight or {name}.weight)")
        parts += [w.ravel(), b.reshape(cout)]
    return np.concatenate(parts).astype(np.float32)


def load_weights(path: str, variant: int) -> np.ndarray:
    """Flat f32 array from a local Ultralytics checkpoint (state_dict keys,
    fused or unfused; see read_state_dict for the accepted formats)."""
    return flat_from_state_dict(read_state_dict(path), variant)


DTYPES = {"bf16": 0, "fp8": 1}  # RV_YOLO_DTYPE_BF16 / RV_YOLO_DTYPE_FP8


def pack(variant: int, flat: np.ndarray, dtype: str = "bf16") -> np.ndarray:
    """Device layout as a u8 host array: bf16 [Cout16][ky][kx][Cin32] + f32
    bias, or (dtype 'fp8') OCP e4m3 [Cout16][ky][kx][Cin64] + f32 bias + f32
    per-cout power-of-two scales for every conv the fp8 plan runs in fp8."""
    lib = _lib.load()
    dt = DTYPES[dtype]
    flat = np.ascontiguousarray(flat, np.float32)
    nbytes = lib.rv_yolo_packed_bytes2(variant, dt)
    out = np.zeros(nbytes, np.uint8)
    _lib.check(lib.rv_yolo_pack2(variant, dt, flat.ctypes.data, flat.size, out.ctypes.data, nbytes),
               "rv_yolo_pack2")
    return out


def weights_from_config(det_cfg: dict, variant: int) -> np.ndarray:
    """The detector's weights for a detect config (default.yaml:38-45 keys):
    ``weights: <path>`` loads a local Ultralytics state_dict (load_weights);
    ``weights: synthetic`` opts in to the seeded synthetic weights (``seed``).
    With no ``weights`` key the synthetic weights are used too, with a
    warning: the reference's YOLO(model) loads the real checkpoint, and a
    production run must not silently detect with random weights."""
    import warnings
    w = det_cfg.get("weights")
    seed = int(det_cfg.get("seed", 0))
    if w and str(w).lower() != "synthetic":
        return load_weights(str(w), variant)
    if not w:
        warnings.warn(f"detect.model={det_cfg.get('model', 'yolov8n.pt')!r} but no detect.weights "
                      "file is configured: using seeded SYNTHETIC weights (set detect.weights to "
                      "a local state_dict, or to 'synthetic' to silence this)", RuntimeWarning,
                      stacklevel=2)
    return synthetic_weights(variant, seed=seed)
