"""rvs_amd -- MI355X-native (gfx950) road-vision hot path.

Drop-in for the plugin surfaces of YJxyzxyz/road-vision-system:
  preprocess  (src/preprocess: PreprocessPipeline, op REGISTRY)
  detect      (src/detect: Detection, Detector, build_detector)
  track       (src/track: Tracker, build_tracker)
  geometry    (src/geometry: GroundProjector, HomographyProjector, build_projector)
backed by the hand-written HIP kernels of librvhip.so (include/rvhip.h).
"""
__version__ = "0.1.0"
