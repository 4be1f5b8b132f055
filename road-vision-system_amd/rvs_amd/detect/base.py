"""Detector interface (mirrors src/detect/base.py:6-13)."""
from abc import ABC, abstractmethod
from typing import List

import numpy as np

from .types import Detection


class Detector(ABC):
    @abstractmethod
    def infer(self, bgr: np.ndarray) -> List[Detection]:
        """BGR uint8 (H,W,3) -> detections."""
        raise NotImplementedError()

    def close(self):
        pass
