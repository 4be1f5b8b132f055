"""Capture front end (src/io_video)."""
from .capture import Frame, MultiStreamCapture, VideoSource, write_y4m

__all__ = ["Frame", "MultiStreamCapture", "VideoSource", "write_y4m"]
