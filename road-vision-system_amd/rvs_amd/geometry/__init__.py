from .projector import GroundProjector, HomographyProjector, build_projector, find_homography

__all__ = ["GroundProjector", "HomographyProjector", "build_projector", "find_homography"]
