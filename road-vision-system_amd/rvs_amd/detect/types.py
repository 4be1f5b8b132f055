"""Detection result type -- field-for-field the reference's
src/detect/types.py:4-15."""
from dataclasses import dataclass
from typing import Optional


@dataclass
class Detection:
    x1: float
    y1: float
    x2: float
    y2: float
    conf: float
    cls_id: int
    cls_name: str
    track_id: Optional[int] = None
    distance_m: Optional[float] = None
    speed_kmh: Optional[float] = None
