"""Config loading (mirrors src/config.py:5-108): the same defaults dict,
deep-merged with a YAML file; None sections become {}.  The default file is
configs/default.yaml shipped with this package (the reference's values)."""
from __future__ import annotations

import os
from copy import deepcopy
from pathlib import Path

import yaml

_DEFAULTS = {
    "camera": {"source": 0, "width": 1280, "height": 720, "fps_request": 30, "backend": "auto"},
    "preview": {"show_fps": True,
                "compare": {"enable": True, "layout": "h", "label_raw": "RAW",
                            "label_proc": "PROC", "divider_px": 4},
                "record": {"enable": False, "path": "out_compare.mp4", "fps": 30}},
    "preprocess": {"enabled": False, "chain": [],
                   "auto_gate": {"enable_low_contrast_gate": False, "contrast_thresh": 20.0}},
    "detect": {"enabled": False, "backend": "ultralytics", "model": "yolov8n.pt",
               "device": "auto", "conf_thres": 0.25, "iou_thres": 0.7, "max_det": 100,
               "classes_keep": []},
    "tracking": {"enabled": False, "backend": "sort", "max_staleness": 1.0, "min_hits": 3,
                 "iou_threshold": 0.3, "speed_window": 0.75},
    "geometry": {"enabled": False,
                 "projector": {"type": "homography", "image_points": [], "world_points": [],
                               "origin": [0.0, 0.0], "max_distance": 1_000_000.0}},
    "vis": {"draw": {"det": True, "thickness": 2, "font_scale": 0.6}},
}

DEFAULT_YAML = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs", "default.yaml")


def _merge(a: dict, b: dict):
    out = deepcopy(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = v
    return out


def _none_to_dict(x):
    if x is None:
        return {}
    if isinstance(x, dict):
        return {k: _none_to_dict(v) for k, v in x.items()}
    return x


def load_config(path: str | None = None) -> dict:
    cfg_path = Path(path) if path else Path(DEFAULT_YAML)
    if not cfg_path.exists():
        raise FileNotFoundError(f"config not found: {cfg_path}")
    with open(cfg_path, "r", encoding="utf-8") as f:
        user = yaml.safe_load(f) or {}
    return _merge(_DEFAULTS, _none_to_dict(user))
