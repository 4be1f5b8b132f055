"""Fog + rain synthetic frames on the GPU.

Mirrors ``EnhancedFogSynthesizer`` (src/augment/fog.py:84-299): same
constructor arguments, same presets (fog.py:73-77), ``synthesize(bgr)`` ->
``(hazy_u8, meta)``, and the parameters are drawn from
``np.random.RandomState(seed)`` in the reference's order (fog.py:245-291).
``synthesize_batch`` fogs a (B, H, W, 3) device batch, one parameter draw
per frame (tools/fog_batch.py:7-34 is the offline driver the reference has
for this).

Two device paths:
  * ``filters=True`` (default, the reference's synthesize): rv_fog_full_u8
    runs every stage -- depth proxy, value-noise beta map, the image
    airlight (band luminance quantile, masked mean, tint, filtered gradient
    map, fog.py:120-139), the edge-guided transmission (the bilateral
    fallback of _guided_filter that opencv-python runs, fog.py:55-67),
    scattering + veil, glow, depth blur, local contrast fade, tint, gamma and
    the sensor-noise normals the draw produced (fog.py:182-293).
  * ``filters=False``: rv_fog_rain_u8, the one-pass scattering core (depth,
    beta map, airlight gradient around a neutral sky, scattering, veil,
    tint, gamma); the config-5 parity tests pin their inputs with it.
Rain streaks (rain_p > 0) are an addition on both paths: the reference has
fog only.
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
NPARAM_FULL, NFULL = 24, 8  # include/rvhip.h RV_FOG_NPARAM_FULL / RV_FOG_NFULL
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


def fog_depth(h: int, w: int, y_h_ratio=0.42, vanishing_x_ratio=0.5, sky_boost=1.25,
              road_damp=0.9, horizon_softness=0.06) -> np.ndarray:
    """_depth_proxy's clipped depth map (fog.py:141-164), f32 (h, w), with
    numpy's f32 operations in the reference's order."""
    y_h = int(y_h_ratio * h)
    yy, xx = np.arange(h, dtype=_F), np.arange(w, dtype=_F)
    dp = _F(1) / np.maximum(yy - _F(y_h), _F(1))
    dp = _F(0.7) * (dp / dp.max())
    vx, vy = _F(vanishing_x_ratio * w), _F(y_h)
    dxx, dyy = xx[None, :] - vx, yy[:, None] - vy
    dv = _F(1) / (np.sqrt(dxx * dxx + dyy * dyy) + _F(1))
    d = dp[:, None] + _F(0.3) * (dv / dv.max())
    dmin = d.min()
    d = (d - dmin) / max(_F(1e-6), d.max() - dmin)
    soft = _F(max(1e-3, horizon_softness) * h)
    sw = _F(1) / (_F(1) + np.exp(-((_F(y_h) - yy) / soft)))
    fac = (_F(1) + _F(sky_boost - 1.0) * sw) * np.power(_F(road_damp), _F(1) - sw)
    return np.clip(d * fac[:, None], _F(0), _F(1)).astype(_F)


DEPTH_BANDS = (0.33, 0.66, 1.0)  # _depth_blur's bands (fog.py:199)


def depth_band_map(depth: np.ndarray) -> np.ndarray:
    """u8 map: the _depth_blur band (0, 1, 2) each pixel's mask belongs to,
    3 for none (depth == 1), with the reference's f32 comparisons."""
    out = np.full(depth.shape, 3, np.uint8)
    prev = np.zeros_like(depth)
    for i, b in enumerate(DEPTH_BANDS):
        out[(depth >= prev) & (depth < b)] = i
        prev = np.full_like(depth, b)
    return out


def band_radii(depth: np.ndarray, bands: np.ndarray, beta: float, depth_blur_max: float):
    """_depth_blur's per-band Gaussian size for one frame (fog.py:195-209):
    rad (odd, > 1) or 0 where the band is skipped."""
    r = np.clip(depth * depth_blur_max * (0.5 + beta), 0.0, depth_blur_max * 1.5)
    out = []
    for i in range(3):
        m = bands == i
        if m.astype(_F).sum() < 100:
            out.append(0)
            continue
        rad = int(max(1, np.mean(r[m]) * 1.5)) | 1
        out.append(rad if rad > 1 else 0)
    return out


def airlight_unit_map(h: int, w: int, radius: int = 16, sigma: float = 12.0) -> np.ndarray:
    """The airlight map's filter on the unit gradient map vgrad x xgrad
    (fog.py:132-138): bilateralFilter(d = 2*16+1, sigma 12, 12) on a map whose
    values differ by < 0.25 is its normalised spatial disk filter to < 1e-5
    (colour weights >= 0.9998), and the disk filter of a separable map is a
    sum of rank-1 terms: per row offset dy, the row filter of xgrad over
    |dx| <= floor(sqrt(r^2 - dy^2)) (BORDER_REFLECT_101), scaled by
    g(dy) vgrad(y + dy).  float64, returned as f32 (h, w)."""
    vg = np.linspace(1.0, 0.85, h, dtype=_F).astype(np.float64)
    xg = np.linspace(0.95, 1.05, w, dtype=_F).astype(np.float64)

    def refl(i, n):
        i = np.abs(i)
        return np.abs(np.where(i >= n, 2 * n - 2 - i, i))
    c = -0.5 / (sigma * sigma)
    ys, xs = np.arange(h), np.arange(w)
    num = np.zeros((h, w))
    den = 0.0
    for dy in range(-radius, radius + 1):
        row = np.zeros(w)
        wsum = 0.0
        for dx in range(-radius, radius + 1):
            r2 = dy * dy + dx * dx
            if r2 > radius * radius:
                continue
            g = float(np.float32(np.exp(r2 * c)))
            row += g * xg[refl(xs + dx, w)]
            wsum += g
        num += vg[refl(ys + dy, h)][:, None] * row[None, :]
        den += wsum
    return (num / den).astype(_F)


def quantile_consts(n: int, q: float = 0.9):
    """np.quantile(f32 array of n, q) 'linear' constants: q is cast to the
    array's f32, the virtual index (n-1)*q is f32, k its floor and t the f32
    remainder (numpy/lib/_function_base_impl.py _quantile / _lerp)."""
    vi = _F(n - 1) * _F(q)
    k = int(np.floor(vi))
    return k, float(_F(vi - _F(k)))


class FogSynthesizer:
    """Drop-in for EnhancedFogSynthesizer (fog.py:84-117) on the GPU.

    filters=True (default) runs the reference's whole synthesize
    (rv_fog_full_u8); filters=False the one-pass scattering core
    (rv_fog_rain_u8).  The draw order is the reference's either way."""

    def __init__(self, level: str = "medium", mor: Optional[float] = None,
                 y_h_ratio: float = 0.42, vanishing_x_ratio: float = 0.5,
                 perlin_scale_ratio: float = 0.18, perlin_octaves: int = 2,
                 sky_boost: float = 1.25, road_damp: float = 0.9, edge_guided: bool = True,
                 horizon_softness: float = 0.06, depth_blur_max: float = 3.5,
                 global_veil: float = 0.06, seed: Optional[int] = None,
                 rain_p: float = 0.0, rain_len: int = 16, device="cuda", filters: bool = True):
        if level not in FOG_PRESETS:
            raise KeyError(level)  # FOG_PRESETS[self.level], fog.py:245
        if not 1 <= int(perlin_octaves) <= MAX_OCT:
            raise ValueError(f"perlin_octaves must be in [1, {MAX_OCT}]")
        self.level, self.mor = level, mor
        self.y_h_ratio, self.vx_ratio = y_h_ratio, vanishing_x_ratio
        self.perlin_scale_ratio, self.perlin_octaves = perlin_scale_ratio, int(perlin_octaves)
        self.sky_boost, self.road_damp = sky_boost, road_damp
        self.edge_guided, self.horizon_softness = edge_guided, horizon_softness
        self.depth_blur_max, self.global_veil = depth_blur_max, global_veil
        self.rain_p, self.rain_len = float(rain_p), int(rain_len)
        self.filters = bool(filters)
        self.rng = np.random.RandomState(seed) if seed is not None else np.random
        self.device = torch.device(device)
        self._scenes: Dict[Tuple[int, int], tuple] = {}
        self._full: Dict[Tuple[int, int], dict] = {}
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
            for gh, gw, _ in octs:  # noise sample taps (rand_perlin, fog.py:22-29)
                for n, gn in ((h, gh), (w, gw)):
                    s = (np.arange(n) * gn).astype(_F) / _F(n)
                    i0 = np.floor(s)
                    taps += [i0, np.minimum(i0 + 1, gn).astype(_F), (s - i0).astype(_F)]
            scene = torch.from_numpy(np.concatenate([rows.ravel(), cols] + taps)
                                     .astype(_F)).to(self.device)
            self._scenes[key] = (consts, scene, octs, stride)
        return self._scenes[key]

    def _full_scene(self, h: int, w: int) -> dict:
        """The full path's per-resolution maps: clipped depth, depth-band
        map, the airlight unit map, and the band quantile constants."""
        key = (h, w)
        if key not in self._full:
            depth = fog_depth(h, w, self.y_h_ratio, self.vx_ratio, self.sky_boost,
                              self.road_damp, self.horizon_softness)
            bands = depth_band_map(depth)
            band_h = max(10, int(0.12 * h))  # fog.py:122
            k, t = quantile_consts(band_h * w)
            full = np.zeros(NFULL, _F)
            full[:4] = [band_h, k, t, 1.0 if self.edge_guided else 0.0]
            dev = self.device
            self._full[key] = dict(
                depth=depth, bands=bands, full=full,
                depth_d=torch.from_numpy(depth).to(dev),
                bands_d=torch.from_numpy(bands).to(dev),
                amap_d=torch.from_numpy(airlight_unit_map(h, w)).to(dev))
        return self._full[key]

    # --- one frame's random draws, in fog.py's order ---
    def draw(self, h: int, w: int):
        """One frame's draws: (params f32[NPARAM], noise grids) for the core
        path, (params f32[NPARAM_FULL], noise grids, sensor-noise normals or
        None) for the full path."""
        consts, _, octs, stride = self._scene(h, w)
        rng = self.rng
        if self.mor is not None and self.mor > 0:  # fog.py:239-244
            base_beta = 3.912 / float(self.mor)
            glow_rng, cdrop_rng, a_rng = (0.12, 0.45), (0.08, 0.22), (0.86, 0.98)
        else:  # fog.py:245-250
            p = FOG_PRESETS[self.level]
            base_beta = _rand_range(*p["beta"], rng)
            glow_rng, cdrop_rng, a_rng = p["glow"], p["contrast_drop"], p["airlight"]
        # _beta_map -> rand_perlin(seed=rng.randint(1e9)) (fog.py:166-169, 8-27)
        prng = np.random.RandomState(rng.randint(1e9))
        grids = np.concatenate([prng.rand(gh + 1, gw + 1).astype(_F).ravel()
                                for gh, gw, _ in octs])
        tint_a = rng.uniform(-0.02, 0.02, size=3).astype(_F)  # fog.py:129
        a_target = _rand_range(*a_rng, rng)  # fog.py:257
        glow = _rand_range(*glow_rng, rng)  # fog.py:273
        cdrop = _rand_range(*cdrop_rng, rng)  # fog.py:280
        tint = (1.0 + rng.uniform(-0.015, 0.02, size=3)).astype(_F)  # fog.py:284
        gamma = 1.0
        if rng.rand() < 0.35:  # fog.py:286-288
            gamma = 1.0 + rng.uniform(-0.04, 0.05)
        noise = None
        if rng.rand() < 0.3:  # sensor noise (fog.py:289-291)
            noise = rng.normal(0, 0.0035, size=(h, w, 3)).astype(_F)
        rain_seed = rng.randint(1 << 24) if self.rain_p > 0 else 0
        if not self.filters:
            # core path: airlight around a neutral sky; the A_map scale to the
            # preset mean uses the separable gradient map's mean (fog.py:257)
            a_rgb = np.clip(_F(0.9) + tint_a, _F(0.7), _F(1.0)).astype(_F)
            a_mean = float(np.mean(a_rgb.astype(np.float64))) * 0.925 * 1.0
            params = np.zeros(NPARAM, _F)
            params[:10] = [base_beta, a_rgb[0], a_rgb[1], a_rgb[2], a_target / max(1e-6, a_mean),
                           tint[0], tint[1], tint[2], gamma, rain_seed]
            return params, grids
        fs = self._full_scene(h, w)
        k = int(9 + 20 * glow) | 1  # fog.py:186
        k2 = int(max(7, (h + w) * (0.003 + 0.01 * glow))) | 1  # fog.py:189
        d = int(5 + cdrop * 20) | 1  # fog.py:220
        if max(k, k2) > 63 or d > 15:
            raise ValueError(f"filter sizes k={k} k2={k2} d={d} exceed the device limits "
                             "(63 / 15)")
        rads = band_radii(fs["depth"], fs["bands"], base_beta, self.depth_blur_max)
        if max(rads) > 63:
            raise ValueError(f"depth-blur kernel {max(rads)} exceeds 63")
        params = np.zeros(NPARAM_FULL, _F)
        params[:21] = [base_beta, tint_a[0], tint_a[1], tint_a[2], a_target, tint[0], tint[1],
                       tint[2], gamma, rain_seed, glow, cdrop, 0.0 if noise is None else 1.0,
                       rads[0], rads[1], rads[2], k, k2, d, 0.0, 0.0]
        return params, grids, noise

    def prepare(self, draws):
        """Upload a list of per-frame draws once: (params, grids[, noise]) on
        device (noise is None when no frame drew sensor noise)."""
        params = torch.from_numpy(np.stack([d[0] for d in draws])).to(self.device)
        grids = torch.from_numpy(np.stack([d[1] for d in draws])).to(self.device)
        if len(draws[0]) == 2:
            return params, grids
        noise = None
        if any(d[2] is not None for d in draws):
            shp = next(d[2] for d in draws if d[2] is not None).shape
            noise = torch.from_numpy(np.stack([d[2] if d[2] is not None else
                                               np.zeros(shp, _F) for d in draws])).to(self.device)
        return params, grids, noise

    def synthesize_batch(self, frames: torch.Tensor, out: Optional[torch.Tensor] = None,
                         draws=None, prepared=None) -> torch.Tensor:
        """(B, H, W, 3) u8 device frames -> fogged copy; one draw per frame
        (or the given list of draws, or tensors from prepare())."""
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
        params, grids = prepared[0], prepared[1]
        npar = NPARAM_FULL if self.filters else NPARAM
        if len(prepared) != (3 if self.filters else 2) or params.shape != (B, npar) or \
                grids.shape != (B, stride) or params.device != x.device or \
                grids.device != x.device:
            raise ValueError("prepared draws do not match the batch / path")
        lib = _lib.load()
        if not self.filters:
            need = max(int(lib.rv_fog_ws_bytes(B)), 8)
        else:
            need = max(int(lib.rv_fog_full_ws_bytes(B, H, W)), 8)
        if self._ws is None or self._ws.numel() < need or self._ws.device != x.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
        if not self.filters:
            call("rv_fog_rain_u8", ptr(x), ptr(out), B, H, W, pitch, consts.ctypes.data, NCONST,
                 ptr(scene), ptr(params), ptr(grids), stride, ptr(self._ws), self._ws.numel(),
                 stream_ptr())
            return out
        fs = self._full_scene(H, W)
        noise = prepared[2]
        if noise is not None and (noise.shape != (B, H, W, 3) or noise.device != x.device):
            raise ValueError("sensor-noise batch does not match the frames")
        call("rv_fog_full_u8", ptr(x), ptr(out), B, H, W, pitch, consts.ctypes.data, NCONST,
             fs["full"].ctypes.data, NFULL, ptr(scene), ptr(fs["depth_d"]), ptr(fs["amap_d"]),
             ptr(fs["bands_d"]), ptr(params), ptr(grids), stride, ptr(noise), ptr(self._ws),
             self._ws.numel(), stream_ptr())
        return out

    def synthesize(self, bgr_uint8, level: Optional[str] = None):
        """fog.py:227: BGR u8 (numpy or device tensor) -> (hazy u8, meta)."""
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
        H, W = x.shape[-3], x.shape[-2]
        meta = {"beta": float(p[0]), "tint": p[5:8].copy(), "gamma": float(p[8]),
                "y_h": int(self.y_h_ratio * H), "consts": self._scene(H, W)[0]}
        if self.filters:
            fs = self._full_scene(H, W)
            meta.update({"airlight_tint": p[1:4].copy(), "airlight_target": float(p[4]),
                         "glow": float(p[10]), "contrast_drop": float(p[11]),
                         "depth": fs["depth"], "depth_blur_rad": [int(v) for v in p[13:16]]})
        else:
            meta.update({"A_rgb": p[1:4].copy(), "A_scale": float(p[4])})
        return (y.cpu().numpy() if was_np else y), meta


def _rand_range(lo, hi, rng) -> float:  # fog.py:79-80
    return float(lo + (hi - lo) * rng.rand())


