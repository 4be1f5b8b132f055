"""Fog + rain synthetic frames on the GPU.

Mirrors ``EnhancedFogSynthesizer`` (src/augment/fog.py:84-299): same
constructor arguments, same presets (fog.py:73-77), ``synthesize(bgr)`` ->
``(hazy_u8, meta)``, and the parameters are drawn from
``np.random.RandomState(seed)`` in the reference's order (fog.py:251-293).
The per-pixel work runs in one HIP pass (``rv_fog_rain_u8``,
csrc/augment.hip); ``synthesize_batch`` fogs a (B, H, W, 3) device batch, one
parameter draw per frame (tools/fog_batch.py:7-34 is the offline driver the
reference has for this).

Restated subset (DESIGN.md "Fog generator"): depth proxy (fog.py:141-163),
value-noise beta map (fog.py:8-45,166-169), transmission without the guided
filter (fog.py:172-173), airlight as the reference's vertical x horizontal
gradient map around a neutral sky colour (fog.py:128-134; the image quantile
and guided filter are not restated), scattering and global veil
(fog.py:271-275), tint and gamma (fog.py:291-294).  Glow, depth blur, local
contrast fade and sensor noise are OpenCV filters/normal draws that the
config-5 workload does not need; their random draws are still consumed
(except the H x W x 3 sensor-noise normals) so the parameter stream follows
the reference's order.  Rain streaks (rain_p > 0) are an addition: the
reference has fog only.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .. import _lib
from .._lib import call, ptr, stream_ptr

FOG_PRESETS = {  # fog.py:73-77
    "light": dict(beta=(0.03, 0.06), airlight=(0.82, 0.93), glow=(0.12, 0.22),
                  contrast_drop=(0.06, 0.12)),
    "medium": dict(beta=(0.06, 0.12), airlight=(0.86, 0.96), glow=(0.18, 0.34),
                   contrast_drop=(0.10, 0.18)),
    "heavy": dict(beta=(0.12, 0.22), airlight=(0.90, 0.99), glow=(0.28, 0.48),
                  contrast_drop=(0.15, 0.26)),
}

NCONST, NPARAM, MAX_OCT = 26, 16, 4
_F = np.float32


def perlin_octaves(h: int, w: int, scale: int, octaves: int = 2, persistence: float = 0.5,
                   lacunarity: float = 2.0):
    """[(gh, gw, amp)] and norm of rand_perlin's octaves (fog.py:12-21)."""
    freq, amp, norm, out = 1.0 / max(1, scale), 1.0, 0.0, []
    for _ in range(max(1, octaves)):
        out.append((max(1, int(h * freq)), max(1, int(w * freq)), amp))
        norm += amp
        amp *= persistence
        freq *= lacunarity
    return out, norm


def fog_scene(h: int, w: int, y_h_ratio=0.42, vanishing_x_ratio=0.5, sky_boost=1.25,
              road_damp=0.9, horizon_softness=0.06, global_veil=0.06):
    """Resolution-only terms of _depth_proxy (fog.py:141-163), the veil weight
    (fog.py:274) and the airlight gradients (fog.py:132-133), in f32.
    Returns (consts-prefix dict, rows (4, h), cols (w,))."""
    y_h = int(y_h_ratio * h)
    yy = np.arange(h, dtype=_F)
    xx = np.arange(w, dtype=_F)
    dp = _F(1) / np.maximum(yy - _F(y_h), _F(1))
    row_dp = _F(0.7) * (dp / dp.max())
    vx, vy = _F(vanishing_x_ratio * w), _F(y_h)
    dx, dy = xx[None, :] - vx, yy[:, None] - vy
    dv = _F(1) / (np.sqrt(dx * dx + dy * dy) + _F(1))
    dv_max = dv.max()
    d = row_dp[:, None] + _F(0.3) * (dv / dv_max)
    d_min = d.min()
    d_range = max(_F(1e-6), d.max() - d_min)
    softness = _F(max(1e-3, horizon_softness) * h)
    sw = (_F(1) / (_F(1) + np.exp(-((_F(y_h) - yy) / softness)))).astype(_F)
    fac = ((_F(1) + _F(sky_boost - 1.0) * sw) * np.power(_F(road_damp), _F(1) - sw)).astype(_F)
    gv = (_F(global_veil) * (_F(0.6) + _F(0.4) * sw)).astype(_F)
    vgrad = np.linspace(1.0, 0.85, h, dtype=_F)
    xgrad = np.linspace(0.95, 1.05, w, dtype=_F)
    rows = np.stack([row_dp, fac, gv, vgrad]).astype(_F)
    return dict(vx=vx, vy=vy, dv_max=dv_max, d_min=d_min, d_range=d_range, y_h=y_h), rows, xgrad


class FogSynthesizer:
    """Drop-in for EnhancedFogSynthesizer (fog.py:84-116) on the GPU."""

    def __init__(self, level: str = "medium", mor: Optional[float] = None,
                 y_h_ratio: float = 0.42, vanishing_x_ratio: float = 0.5,
                 perlin_scale_ratio: float = 0.18, perlin_octaves: int = 2,
                 sky_boost: float = 1.25, road_damp: float = 0.9, edge_guided: bool = True,
                 horizon_softness: float = 0.06, depth_blur_max: float = 3.5,
                 global_veil: float = 0.06, seed: Optional[int] = None,
                 rain_p: float = 0.0, rain_len: int = 16, device="cuda"):
        if level not in FOG_PRESETS:
            raise KeyError(level)  # FOG_PRESETS[self.level], fog.py:255
        if not 1 <= int(perlin_octaves) <= MAX_OCT:
            raise ValueError(f"perlin_octaves must be in [1, {MAX_OCT}]")
        self.level, self.mor = level, mor
        self.y_h_ratio, self.vx_ratio = y_h_ratio, vanishing_x_ratio
        self.perlin_scale_ratio, self.perlin_octaves = perlin_scale_ratio, int(perlin_octaves)
        self.sky_boost, self.road_damp = sky_boost, road_damp
        self.edge_guided, self.horizon_softness = edge_guided, horizon_softness
        self.depth_blur_max, self.global_veil = depth_blur_max, global_veil
        self.rain_p, self.rain_len = float(rain_p), int(rain_len)
        self.rng = np.random.RandomState(seed) if seed is not None else np.random
        self.device = torch.device(device)
        self._scenes: Dict[Tuple[int, int], tuple] = {}
        self._ws: Optional[torch.Tensor] = None
        self.last_draws = None

    # --- per-resolution constants (cached) ---
    def _scene(self, h: int, w: int):
        key = (h, w)
        if key not in self._scenes:
            sc, rows, cols = fog_scene(h, w, self.y_h_ratio, self.vx_ratio, self.sky_boost,
                                       self.road_damp, self.horizon_softness, self.global_veil)
            octs, norm = perlin_octaves(h, w, max(16, int(self.perlin_scale_ratio * w)),
                                        self.perlin_octaves)
            consts = np.zeros(NCONST, _F)
            consts[:9] = [sc["vx"], sc["vy"], sc["dv_max"], sc["d_min"], sc["d_range"], 0.0,
                          self.rain_p, self.rain_len, len(octs)]
            for j, (gh, gw, amp) in enumerate(octs):
                consts[9 + 4 * j:12 + 4 * j] = [gh, gw, amp]
            consts[25] = norm
            stride = sum((gh + 1) * (gw + 1) for gh, gw, _ in octs)
            taps = []
            for gh, gw, _ in octs:  # noise sample taps (rand_perlin, fog.py:24-31)
                for n, gn in ((h, gh), (w, gw)):
                    s = (np.arange(n) * gn).astype(_F) / _F(n)
                    i0 = np.floor(s)
                    taps += [i0, np.minimum(i0 + 1, gn).astype(_F), (s - i0).astype(_F)]
            scene = torch.from_numpy(np.concatenate([rows.ravel(), cols] + taps)
                                     .astype(_F)).to(self.device)
            self._scenes[key] = (consts, scene, octs, stride)
        return self._scenes[key]

    # --- one frame's random draws, in fog.py's order ---
    def draw(self, h: int, w: int) -> Tuple[np.ndarray, np.ndarray]:
        """(params f32[NPARAM], noise grids f32[grid_stride]) for one frame."""
        consts, _, octs, stride = self._scene(h, w)
        rng = self.rng
        if self.mor is not None and self.mor > 0:  # fog.py:245-250
            base_beta = 3.912 / float(self.mor)
            glow_rng, cdrop_rng, a_rng = (0.12, 0.45), (0.08, 0.22), (0.86, 0.98)
        else:  # fog.py:251-256
            p = FOG_PRESETS[self.level]
            base_beta = _rand_range(*p["beta"], rng)
            glow_rng, cdrop_rng, a_rng = p["glow"], p["contrast_drop"], p["airlight"]
        # _beta_map -> rand_perlin(seed=rng.randint(1e9)) (fog.py:166-169, 8-27)
        prng = np.random.RandomState(rng.randint(1e9))
        grids = np.concatenate([prng.rand(gh + 1, gw + 1).astype(_F).ravel()
                                for gh, gw, _ in octs])
        # _airlight_from_image's tint (fog.py:127), around a neutral sky
        tint_a = rng.uniform(-0.02, 0.02, size=3).astype(_F)
        a_rgb = np.clip(_F(0.9) + tint_a, _F(0.7), _F(1.0)).astype(_F)
        # A_map scale to the preset mean (fog.py:263-264): mean of the
        # separable gradient map, before its clip
        a_mean = float(np.mean(a_rgb.astype(np.float64))) * 0.925 * 1.0
        scale = _rand_range(*a_rng, rng) / max(1e-6, a_mean)
        _rand_range(*glow_rng, rng)  # glow (fog.py:278): drawn, not restated
        _rand_range(*cdrop_rng, rng)  # contrast drop (fog.py:284): drawn, not restated
        tint = (1.0 + rng.uniform(-0.015, 0.02, size=3)).astype(_F)  # fog.py:288
        gamma = 1.0
        if rng.rand() < 0.35:  # fog.py:290-292
            gamma = 1.0 + rng.uniform(-0.04, 0.05)
        if rng.rand() < 0.3:  # sensor noise (fog.py:293-295): not applied, but its
            rng.normal(0, 0.0035, size=(h, w, 3))  # normals advance the stream
            # exactly as the reference's do, so later frames' draws match
        rain_seed = rng.randint(1 << 24) if self.rain_p > 0 else 0
        params = np.zeros(NPARAM, _F)
        params[:10] = [base_beta, a_rgb[0], a_rgb[1], a_rgb[2], scale, tint[0], tint[1],
                       tint[2], gamma, rain_seed]
        return params, grids

    def prepare(self, draws) -> Tuple[torch.Tensor, torch.Tensor]:
        """Upload a list of per-frame draws once: (params, grids) on device."""
        params = torch.from_numpy(np.stack([d[0] for d in draws])).to(self.device)
        grids = torch.from_numpy(np.stack([d[1] for d in draws])).to(self.device)
        return params, grids

    def synthesize_batch(self, frames: torch.Tensor, out: Optional[torch.Tensor] = None,
                         draws=None, prepared=None) -> torch.Tensor:
        """(B, H, W, 3) u8 device frames -> fogged copy; one draw per frame
        (or the given list of (params, grids), or tensors from prepare())."""
        from ..kernels import _frames, _like
        x, B, H, W, pitch = _frames(frames)
        out = _like(x, out)
        consts, scene, octs, stride = self._scene(H, W)
        if prepared is None:
            draws = draws if draws is not None else [self.draw(H, W) for _ in range(B)]
            if len(draws) != B:
                raise ValueError("one draw per frame")
            prepared = self.prepare(draws)
            self.last_draws = draws
        params, grids = prepared
        if params.shape != (B, NPARAM) or grids.shape != (B, stride) or \
                params.device != x.device or grids.device != x.device:
            raise ValueError("prepared draws do not match the batch")
        need = max(int(_lib.load().rv_fog_ws_bytes(B)), 8)
        if self._ws is None or self._ws.numel() < need or self._ws.device != x.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
        call("rv_fog_rain_u8", ptr(x), ptr(out), B, H, W, pitch, consts.ctypes.data, NCONST,
             ptr(scene), ptr(params), ptr(grids), stride, ptr(self._ws), self._ws.numel(),
             stream_ptr())
        return out

    def synthesize(self, bgr_uint8, level: Optional[str] = None):
        """fog.py:239: BGR u8 (numpy or device tensor) -> (hazy u8, meta)."""
        if level is not None:
            if level not in FOG_PRESETS:
                raise KeyError(level)
            self.level = level
        was_np = isinstance(bgr_uint8, np.ndarray)
        x = torch.from_numpy(np.ascontiguousarray(bgr_uint8)).to(self.device) if was_np \
            else bgr_uint8
        y = self.synthesize_batch(x.unsqueeze(0) if x.dim() == 3 else x)
        y = y[0] if x.dim() == 3 else y
        p = self.last_draws[0][0]
        sc = self._scene(x.shape[-3], x.shape[-2])[0]
        meta = {"beta": float(p[0]), "A_rgb": p[1:4].copy(), "A_scale": float(p[4]),
                "tint": p[5:8].copy(), "gamma": float(p[8]), "y_h": int(self.y_h_ratio *
                                                                        x.shape[-3]),
                "consts": sc}
        return (y.cpu().numpy() if was_np else y), meta


def _rand_range(lo, hi, rng) -> float:  # fog.py:79-80
    return float(lo + (hi - lo) * rng.rand())


