from .types import Detection
from .base import Detector
from .registry import build_detector

__all__ = ["Detection", "Detector", "build_detector"]
