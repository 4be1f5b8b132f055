"""PreprocessOp interface (mirrors src/preprocess/base.py:4-16)."""
from abc import ABC, abstractmethod
from typing import Any


class PreprocessOp(ABC):
    """Base class of every preprocess op.

    Contract (identical to the reference): ``__call__(image) -> image`` where
    image is BGR uint8 (H, W, 3).  HIP ops additionally accept a device
    ``torch.Tensor`` shaped (H, W, 3) or (B, H, W, 3) and then return a device
    tensor, so a chain stays resident in HBM.
    """

    def __init__(self, **params: Any):
        self.params = params

    @abstractmethod
    def __call__(self, image):
        pass
