"""Detector factory (mirrors src/detect/registry.py:5-9).

'ultralytics' -- the reference's default backend name (default.yaml:38) --
and 'hip' both resolve to the gfx950 YOLOv8 backend, so an unchanged
reference config drops in."""
from typing import Any, Dict

from .base import Detector


def build_detector(cfg: Dict[str, Any]) -> Detector:
    backend = (cfg.get("backend") or "ultralytics").lower()
    if backend in ("ultralytics", "hip"):
        from .yolo_hip import YOLOHip
        return YOLOHip(cfg)
    raise ValueError(f"unknown detector backend: {backend}")
