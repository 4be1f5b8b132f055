"""HIP preprocess ops (drop-in for src/preprocess/ops/*.py and ops_cuda/*.py).

``CLAHEDehaze`` restates clahe_dehaze.py:13-32 and ``MedianDerain`` restates
median_derain.py:10-14 on the gfx950 kernels of csrc/preprocess.hip.  Parameter
parsing follows the reference line by line (grid clamp, ksize normalisation).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import kernels
from .base import PreprocessOp


def clahe_params(params):
    """(space, clip_limit, grid) exactly as clahe_dehaze.py:14-17 parses them."""
    space = str(params.get("space", "YCrCb")).upper()
    clip_limit = float(params.get("clip_limit", 2.0))
    grid = int(params.get("tile_grid", 8))
    grid = max(2, grid)
    return space, clip_limit, grid


def median_ksize(params):
    """ksize normalisation of median_derain.py:11-13."""
    k = int(params.get("ksize", 3))
    if k % 2 == 0:
        k += 1
    k = max(3, min(k, 9))
    return k


def _to_device(image):
    """np.ndarray (H,W,3) u8 -> (device tensor, was_numpy)."""
    if isinstance(image, torch.Tensor):
        return image, False
    arr = np.ascontiguousarray(image)
    if arr.dtype != np.uint8 or arr.ndim != 3 or arr.shape[2] != 3:
        raise ValueError(f"expected BGR uint8 (H,W,3), got {arr.shape} {arr.dtype}")
    return torch.from_numpy(arr).cuda(), True


def _back(t, was_numpy):
    return t.cpu().numpy() if was_numpy else t


class CLAHEDehaze(PreprocessOp):
    """CLAHE on the luma channel, HIP kernels: YCrCb (default) or LAB
    (clahe_dehaze.py:21-30; any space other than "LAB" takes YCrCb)."""

    def __init__(self, **params):
        super().__init__(**params)
        self.space, self.clip_limit, self.grid = clahe_params(self.params)
        self._ws = None

    def __call__(self, image):
        x, was_np = _to_device(image)
        B = 1 if x.dim() == 3 else x.shape[0]
        need = kernels.clahe_ws_bytes(B, self.grid)
        if self._ws is None or self._ws.numel() < need or self._ws.device != x.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
        fn = kernels.clahe_lab if self.space == "LAB" else kernels.clahe_ycrcb
        out = fn(x, self.grid, self.clip_limit, ws=self._ws)
        return _back(out, was_np)


class MedianDerain(PreprocessOp):
    """Exact k x k median, replicated borders, HIP kernel."""

    def __init__(self, **params):
        super().__init__(**params)
        self.k = median_ksize(self.params)

    def __call__(self, image):
        x, was_np = _to_device(image)
        return _back(kernels.median(x, self.k), was_np)


# The reference registers its OpenCV-CUDA variants under these names
# (src/preprocess/registry.py:19-23); on MI355X they are the same HIP ops.
HIPCLAHEDehaze = CLAHEDehaze
HIPMedianDerain = MedianDerain
CUDACLAHEDehaze = CLAHEDehaze
CUDAMedianDerain = MedianDerain
