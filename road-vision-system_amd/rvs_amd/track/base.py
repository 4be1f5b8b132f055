"""Tracker interface (mirrors src/track/base.py:11-24)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Iterable, List, Optional

from ..detect.types import Detection
from ..geometry import GroundProjector


class Tracker(ABC):
    @abstractmethod
    def update(self, detections: Iterable[Detection], timestamp: float,
               projector: Optional[GroundProjector] = None) -> List[Detection]:
        """Update and return the detections with track_id / distance_m / speed_kmh."""

    def close(self) -> None:
        pass
