"""PreprocessPipeline (mirrors src/preprocess/pipeline.py:7-45).

Same config keys and control flow as the reference: ``enabled``, ``chain``
(list of {name, params}), ``auto_gate`` {enable_low_contrast_gate,
contrast_thresh}.  When the chain is exactly [CLAHEDehaze(YCrCb),
MedianDerain] -- configs/default.yaml:21-31 -- it runs the fused HIP pass
(rv_clahe_median_u8), which is bit-identical to running the two ops in turn.
"""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from .. import kernels
from .ops import CLAHEDehaze, MedianDerain, _back, _to_device
from .registry import get_op_class


class PreprocessPipeline:
    def __init__(self, config: Dict[str, Any]):
        self.enabled = bool(config.get("enabled", True))
        self.chain_cfg = config.get("chain", []) or []
        self.auto_gate_cfg = config.get("auto_gate", {}) or {}
        self.ops = []
        for node in self.chain_cfg:
            name = node.get("name")
            params = node.get("params", {})
            cls = get_op_class(name)
            self.ops.append(cls(**params))
        # the fused CLAHE+median passes are YCrCb-only; a LAB chain runs op by op
        self._fused = (len(self.ops) == 2 and isinstance(self.ops[0], CLAHEDehaze)
                       and self.ops[0].space != "LAB" and isinstance(self.ops[1], MedianDerain))
        self._ws = None

    def _gate_enabled(self) -> bool:
        return bool(self.auto_gate_cfg.get("enable_low_contrast_gate", False))

    def low_contrast_mask(self, frames: torch.Tensor) -> torch.Tensor:
        """Per-frame `span < contrast_thresh` (pipeline.py:24-30) on device."""
        thresh = float(self.auto_gate_cfg.get("contrast_thresh", 20.0))
        span = kernels.gray_span(frames)
        return span.float() < thresh

    def _run_chain(self, x: torch.Tensor) -> torch.Tensor:
        if self._fused:
            clahe, med = self.ops
            B = 1 if x.dim() == 3 else x.shape[0]
            need = kernels.clahe_ws_bytes(B, clahe.grid)
            if self._ws is None or self._ws.numel() < need or self._ws.device != x.device:
                self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
            if kernels.clahe_median_fits(x, clahe.grid, med.k):
                return kernels.clahe_median(x, clahe.grid, clahe.clip_limit, med.k, ws=self._ws)
            # very fine grids: the LUT window exceeds LDS; the unfused pair
            # gives the identical result.
        out = x
        for op in self.ops:
            out = op(out)
        return out

    def letterbox_fusable(self, H: int, W: int, geo) -> bool:
        """True when the chain is the fused default and the detector's
        LetterBox (geo) can be emitted by the same pass (no gate: the gate
        selects raw frames per frame after the chain)."""
        if not (self.enabled and self._fused) or self._gate_enabled():
            return False
        clahe, med = self.ops
        return kernels.clahe_median_letterbox_fits(H, W, clahe.grid, med.k, geo)

    def run_with_letterbox(self, x: torch.Tensor, geo, lb_out: torch.Tensor,
                           out: torch.Tensor = None):
        """(B,H,W,3) device frames -> (proc, letterboxed proc) in one pass;
        byte-identical to self(x) followed by the detector's letterbox."""
        clahe, med = self.ops
        B = x.shape[0]
        need = kernels.clahe_ws_bytes(B, clahe.grid)
        if self._ws is None or self._ws.numel() < need or self._ws.device != x.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
        return kernels.clahe_median_letterbox(x, clahe.grid, clahe.clip_limit, med.k, geo,
                                              out=out, lb_out=lb_out, ws=self._ws)

    def __call__(self, image, ts: float = None):
        if not self.enabled or not self.ops:
            return image
        x, was_np = _to_device(image)
        if self._gate_enabled():
            low = self.low_contrast_mask(x)
            if x.dim() == 3:
                if not bool(low[0]):
                    return image  # contrast is sufficient -> skip the chain
                return _back(self._run_chain(x), was_np)
            # per frame, as the reference's per-frame loop does: only the
            # low-contrast frames run the chain (gathered into one batch, one
            # host read of the gate); the others pass through unchanged
            sel = torch.nonzero(low).flatten()
            n = int(sel.numel())
            if n == 0:
                return image
            if n == x.shape[0]:
                return _back(self._run_chain(x), was_np)
            out = x.clone()
            out.index_copy_(0, sel, self._run_chain(x.index_select(0, sel).contiguous()))
            return _back(out, was_np)
        return _back(self._run_chain(x), was_np)
