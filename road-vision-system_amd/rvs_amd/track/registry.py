"""Tracker factory (mirrors src/track/registry.py:10-14): 'sort' (the
reference's name) and 'sort_hip' build the gfx950 SORT tracker."""
from typing import Any, Dict

from .base import Tracker


def build_tracker(cfg: Dict[str, Any]) -> Tracker:
    backend = (cfg.get("backend") or "sort").lower()
    if backend in ("sort", "sort_hip"):
        from .sort_hip import SortTracker
        return SortTracker(cfg)
    raise ValueError(f"unknown tracker backend: {backend}")
