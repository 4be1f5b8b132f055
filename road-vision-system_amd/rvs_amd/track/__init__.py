from .base import Tracker
from .registry import build_tracker

__all__ = ["Tracker", "build_tracker"]
