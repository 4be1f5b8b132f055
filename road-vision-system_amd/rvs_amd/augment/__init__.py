"""Synthetic-input augmentation (src/augment in the reference)."""
from .fog import FOG_PRESETS, FogSynthesizer, fog_scene, perlin_octaves

__all__ = ["FOG_PRESETS", "FogSynthesizer", "fog_scene", "perlin_octaves"]
