"""Synthetic-input augmentation (src/augment in the reference)."""
from .fog import (FOG_PRESETS, FogSynthesizer, airlight_unit_map, band_radii, depth_band_map,
                  fog_depth, fog_scene, perlin_octaves, quantile_consts)

__all__ = ["FOG_PRESETS", "FogSynthesizer", "airlight_unit_map", "band_radii", "depth_band_map",
           "fog_depth", "fog_scene", "perlin_octaves", "quantile_consts"]
