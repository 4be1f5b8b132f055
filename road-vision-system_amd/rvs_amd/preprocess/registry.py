"""Name -> op class registry (mirrors src/preprocess/registry.py:14-28)."""
from typing import Dict, Type

from .base import PreprocessOp
from .ops import CLAHEDehaze, MedianDerain

REGISTRY: Dict[str, Type[PreprocessOp]] = {
    "CLAHEDehaze": CLAHEDehaze,
    "MedianDerain": MedianDerain,
    # reference's optional CUDA names and explicit HIP names resolve to the
    # same gfx950 ops
    "CUDACLAHEDehaze": CLAHEDehaze,
    "CUDAMedianDerain": MedianDerain,
    "HIPCLAHEDehaze": CLAHEDehaze,
    "HIPMedianDerain": MedianDerain,
}


def get_op_class(name: str) -> Type[PreprocessOp]:
    if name not in REGISTRY:
        raise KeyError(f"Preprocess op '{name}' not found. Available: {list(REGISTRY.keys())}")
    return REGISTRY[name]
