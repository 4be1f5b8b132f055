"""CPU restatement of the fog + rain generator -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of rv_fog_rain_u8
(csrc/augment.hip) and of the host parameter draw
(rvs_amd/augment/fog.py).  Written independently of both, from the
reference's src/augment/fog.py:
  rand_perlin               fog.py:8-45   (f32 sample positions ys = (y*gh)/h)
  _depth_proxy              fog.py:141-163
  _beta_map                 fog.py:166-169
  _transmission (no filter) fog.py:172-173
  airlight gradient map     fog.py:128-134 (neutral sky 0.9 + tint; no quantile)
  synthesize                fog.py:239-299 (draw order; scattering, veil,
                                            tint, gamma; u8 = int(h*255+.5))
plus the build's rain streaks (hash of (column + y/4, y / rain_len)).

Parity status: the reference's generator needs cv2 (absent) and draws from an
unseeded RNG by default (fog.py:117), so it is not a parity target
(SURVEY §8(f)); this oracle pins the HIP kernel to the build's own stated
restatement.  Tolerance: u8 |d| <= 1 (expf / powf ulp differences between
the device math library and numpy), exact for >= 99 % of channel values.
"""
from __future__ import annotations

import numpy as np

F = np.float32
PRESETS = {  # fog.py:73-77
    "light": ((0.03, 0.06), (0.82, 0.93), (0.12, 0.22), (0.06, 0.12)),
    "medium": ((0.06, 0.12), (0.86, 0.96), (0.18, 0.34), (0.10, 0.18)),
    "heavy": ((0.12, 0.22), (0.90, 0.99), (0.28, 0.48), (0.15, 0.26)),
}


def octaves(h, w, scale_ratio=0.18, n=2):
    scale = max(16, int(scale_ratio * w))  # fog.py:167
    freq, amp, res, norm = 1.0 / max(1, scale), 1.0, [], 0.0
    for _ in range(max(1, n)):  # fog.py:17-41
        res.append((max(1, int(h * freq)), max(1, int(w * freq)), amp))
        norm += amp
        amp *= 0.5
        freq *= 2.0
    return res, norm


def draw(rng, h, w, level="medium", mor=None, scale_ratio=0.18, n_oct=2, rain=False):
    """One frame's parameters in synthesize()'s draw order (fog.py:245-293)."""
    if mor is not None and mor > 0:
        beta = 3.912 / float(mor)
        beta_r, a_r, glow_r, cd_r = None, (0.86, 0.98), (0.12, 0.45), (0.08, 0.22)
    else:
        beta_r, a_r, glow_r, cd_r = PRESETS[level]
        beta = beta_r[0] + (beta_r[1] - beta_r[0]) * rng.rand()
    octs, _ = octaves(h, w, scale_ratio, n_oct)
    g = np.random.RandomState(rng.randint(1e9))
    grids = [g.rand(gh + 1, gw + 1).astype(F) for gh, gw, _ in octs]
    a_rgb = np.clip(F(0.9) + rng.uniform(-0.02, 0.02, size=3).astype(F), F(0.7), F(1.0))
    a_target = a_r[0] + (a_r[1] - a_r[0]) * rng.rand()
    a_scale = a_target / max(1e-6, float(np.mean(a_rgb.astype(np.float64))) * 0.925)
    rng.rand()  # glow
    rng.rand()  # contrast drop
    tint = (1.0 + rng.uniform(-0.015, 0.02, size=3)).astype(F)
    gamma = 1.0 + rng.uniform(-0.04, 0.05) if rng.rand() < 0.35 else 1.0
    noise = rng.rand() < 0.3  # sensor-noise coin (fog.py:293-295)
    if noise:  # not applied, but its normals advance the stream
        rng.normal(0, 0.0035, size=(h, w, 3))
    seed = rng.randint(1 << 24) if rain else 0
    return dict(beta=F(beta), a_rgb=a_rgb.astype(F), a_scale=F(a_scale), tint=tint,
                gamma=F(gamma), rain_seed=int(seed), grids=grids, sensor_noise=bool(noise))


def _lowbias32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def noise(h, w, grids, octs, norm):
    """rand_perlin before its min/max normalisation (fog.py:24-42), f32."""
    yy, xx = np.arange(h), np.arange(w)
    base = np.zeros((h, w), F)
    for g, (gh, gw, amp) in zip(grids, octs):
        ys = (yy * gh).astype(F) / F(h)
        xs = (xx * gw).astype(F) / F(w)
        y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
        y1, x1 = np.minimum(y0 + 1, gh), np.minimum(x0 + 1, gw)
        wy, wx = (ys - y0.astype(F))[:, None], (xs - x0.astype(F))[None, :]
        g00, g01 = g[y0][:, x0], g[y0][:, x1]
        g10, g11 = g[y1][:, x0], g[y1][:, x1]
        top = g00 * (F(1) - wx) + g01 * wx
        bot = g10 * (F(1) - wx) + g11 * wx
        base = base + F(amp) * (top * (F(1) - wy) + bot * wy)
    return base / F(max(1e-6, norm))


def fog_frame(img, prm, y_h_ratio=0.42, vx_ratio=0.5, sky_boost=1.25, road_damp=0.9,
              softness_ratio=0.06, global_veil=0.06, scale_ratio=0.18, n_oct=2,
              rain_p=0.0, rain_len=16):
    """img (h, w, 3) u8 BGR -> fogged u8, all arithmetic in f32."""
    h, w = img.shape[:2]
    yy, xx = np.arange(h, dtype=F), np.arange(w, dtype=F)
    # _depth_proxy (fog.py:141-163)
    y_h = int(y_h_ratio * h)
    dp = F(1) / np.maximum(yy - F(y_h), F(1))
    dp = F(0.7) * (dp / dp.max())
    vx, vy = F(vx_ratio * w), F(y_h)
    dxx, dyy = xx[None, :] - vx, yy[:, None] - vy
    dv = F(1) / (np.sqrt(dxx * dxx + dyy * dyy) + F(1))
    d = dp[:, None] + F(0.3) * (dv / dv.max())
    dmin = d.min()
    d = (d - dmin) / max(F(1e-6), d.max() - dmin)
    soft = F(max(1e-3, softness_ratio) * h)
    sw = F(1) / (F(1) + np.exp(-((F(y_h) - yy) / soft)))
    fac = (F(1) + F(sky_boost - 1.0) * sw) * np.power(F(road_damp), F(1) - sw)
    d = np.clip(d * fac[:, None], F(0), F(1))
    # _beta_map (fog.py:166-169) on the normalised noise (fog.py:43)
    octs, norm = octaves(h, w, scale_ratio, n_oct)
    nz = noise(h, w, prm["grids"], octs, norm)
    nn = (nz - nz.min()) / max(F(1e-6), nz.max() - nz.min())
    beta = prm["beta"] * (F(0.85) + F(0.35) * nn)
    t = np.clip(np.exp(-beta * d), F(0.05), F(1))
    # airlight gradient map (fog.py:132-134, 263-264)
    vg = np.linspace(1.0, 0.85, h, dtype=F)[:, None]
    xg = np.linspace(0.95, 1.05, w, dtype=F)[None, :]
    gv = (F(global_veil) * (F(0.6) + F(0.4) * sw))[:, None]
    if rain_p > 0:
        thr = np.uint32(min(float(np.float32(rain_p)) * 4294967296.0, 4294967295.0))
        yi, xi = np.arange(h)[:, None], np.arange(w)[None, :]
        col = (xi + (yi >> 2)).astype(np.uint32)
        seg = np.broadcast_to((yi // int(rain_len)).astype(np.uint32), col.shape)
        hsh = _lowbias32(np.uint32(prm["rain_seed"]) ^
                         _lowbias32(col * np.uint32(0x9E3779B1) + _lowbias32(seg)))
        rain = hsh < thr
    else:
        rain = np.zeros((h, w), bool)
    out = np.empty_like(img)
    for c in range(3):
        A = np.clip(np.clip(prm["a_rgb"][c] * vg * xg, F(0.7), F(1)) * prm["a_scale"],
                    F(0.75), F(1))
        v = img[..., c].astype(F) / F(255)
        hz = v * t + A * (F(1) - t)  # fog.py:271
        hz = np.clip(hz * (F(1) - gv) + A * gv, F(0), F(1))  # fog.py:275
        hz = np.clip(hz * prm["tint"][c], F(0), F(1))  # fog.py:289
        if prm["gamma"] != F(1):
            hz = np.clip(np.power(hz, prm["gamma"]), F(0), F(1))  # fog.py:292
        hz = np.where(rain, hz + (F(1) - hz) * F(0.45), hz)
        out[..., c] = (hz * F(255) + F(0.5)).astype(np.int32).astype(np.uint8)  # fog.py:297
    return out
