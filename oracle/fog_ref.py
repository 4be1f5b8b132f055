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


# ---------------------------------------------------------------------------
# Full synthesize (every filter of fog.py:239-299).  OpenCV is absent, so its
# filters are restated from the OpenCV 4.x sources (scalar forms); parity
# against real OpenCV is unpinned, as for the rest of this module.
#   guided filter    fog.py:55-67   -> the fallback branch opencv-python runs
#                                      (no cv2.ximgproc): bilateralFilter on
#                                      the f32 map, d = 2r+1, sigma 12 / 12
#   image airlight   fog.py:120-139 (band quantile, masked mean, tint,
#                                    gradient map, filter, clip)
#   glow             fog.py:182-192
#   depth blur       fog.py:194-215
#   contrast fade    fog.py:217-225
#   sensor noise     fog.py:289-291 (the draw's own normals are applied)
# ---------------------------------------------------------------------------

def reflect101(idx, n):
    """cv::BORDER_REFLECT_101 (BORDER_DEFAULT) source index."""
    idx = np.asarray(idx)
    if n == 1:
        return np.zeros_like(idx)
    p = np.abs(idx)
    p = np.where(p >= n, 2 * n - 2 - p, p)
    return np.abs(p)


def gray_u8(img):
    """cvtColor BGR2GRAY 8U (RGB2Gray<uchar>, yuv_shift 14)."""
    i = img.astype(np.int32)
    return ((i[..., 0] * 1868 + i[..., 1] * 9617 + i[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


def gaussian_kernel(k, sigma):
    """getGaussianKernel(k, sigma > 0, CV_32F): computed in double, cast."""
    x = np.arange(k, dtype=np.float64) - (k - 1) * 0.5
    t = np.exp((-0.5 / (sigma * sigma)) * x * x)
    return (t * (1.0 / t.sum())).astype(F)


def _sep_pass(img, kern, axis):
    """One symmetric separable pass: s = k_c S_0 + sum_i k_{c+i} (S_-i + S_i)
    in f32 (SymmColumnFilter form), BORDER_REFLECT_101."""
    n = img.shape[axis]
    r = len(kern) // 2
    base = np.arange(n)
    take = lambda off: np.take(img, reflect101(base + off, n), axis=axis)
    s = kern[r] * img
    for i in range(1, r + 1):
        s = s + kern[r + i] * (take(-i) + take(i))
    return s.astype(F)


def gaussian_blur(img, k, sigma):
    """cv2.GaussianBlur(f32, (k, k), sigma): row pass, then column pass."""
    if k <= 1:
        return img.astype(F).copy()
    kern = gaussian_kernel(k, sigma)
    return _sep_pass(_sep_pass(img.astype(F), kern, 1), kern, 0)


def _space_taps(radius, sigma_space, skip_center):
    taps = []
    c = -0.5 / (sigma_space * sigma_space)
    for i in range(-radius, radius + 1):
        for j in range(-radius, radius + 1):
            r = np.sqrt(float(i * i + j * j))
            if r > radius or (skip_center and i == 0 and j == 0):
                continue
            taps.append((i, j, np.float32(np.exp(r * r * c))))
    return taps


def bilateral_f32(src, d, sigma_color, sigma_space):
    """cv::bilateralFilter on a 1-channel CV_32F image (bilateralFilter_32f):
    exp LUT of 4096 bins over the image's value range with linear
    interpolation, the centre tap excluded from the loop and added with
    weight 1, BORDER_REFLECT_101."""
    src = src.astype(F)
    radius = max(d // 2 if d > 0 else int(round(sigma_space * 1.5)), 1)
    mn, mx = float(src.min()), float(src.max())
    if abs(mn - mx) < np.finfo(np.float32).eps:
        return src.copy()
    nb = 1 << 12
    scale_index = F(nb / F(mx - mn))
    lut = np.zeros(nb + 2, F)
    last, cc = F(1), -0.5 / (sigma_color * sigma_color)
    for i in range(nb + 2):
        if last > 0:
            v = i / float(scale_index)
            lut[i] = F(np.exp(v * v * cc))
            last = lut[i]
    h, w = src.shape
    ry, rx = np.arange(h), np.arange(w)
    s = np.zeros_like(src)
    ws = np.zeros_like(src)
    for i, j, sw in _space_taps(radius, sigma_space, True):
        val = src[reflect101(ry + i, h)][:, reflect101(rx + j, w)]
        alpha = np.abs(val - src) * scale_index
        idx = np.floor(alpha).astype(np.int64)
        alpha = alpha - idx.astype(F)
        wgt = sw * (lut[idx] + alpha * (lut[idx + 1] - lut[idx]))
        ws = ws + wgt
        s = s + val * wgt
    return ((s + src) / (ws + F(1))).astype(F)


def bilateral_u8(src, d, sigma_color, sigma_space):
    """cv::bilateralFilter on a 1-channel 8U image (bilateralFilter_8u):
    colour weights per integer |difference|, f32 sums, cvRound(sum / wsum)."""
    radius = max(d // 2 if d > 0 else int(round(sigma_space * 1.5)), 1)
    cw = np.exp(np.arange(256, dtype=np.float64) ** 2 *
                (-0.5 / (sigma_color * sigma_color))).astype(F)
    h, w = src.shape
    ry, rx = np.arange(h), np.arange(w)
    si = src.astype(np.int32)
    s = np.zeros((h, w), F)
    ws = np.zeros((h, w), F)
    for i, j, sw in _space_taps(radius, sigma_space, False):
        val = si[reflect101(ry + i, h)][:, reflect101(rx + j, w)]
        wgt = sw * cw[np.abs(val - si)]
        ws = ws + wgt
        s = s + val.astype(F) * wgt
    return np.rint(s / ws).astype(np.uint8)


def add_weighted_u8(a, alpha, b, beta):
    """cv2.addWeighted 8U: saturate_cast<uchar>(a*alpha + b*beta + 0) in f32."""
    v = a.astype(F) * F(alpha) + b.astype(F) * F(beta)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def airlight_rgb(img_f):
    """_airlight_from_image's sky colour before the tint (fog.py:120-127)."""
    h = img_f.shape[0]
    band_h = max(10, int(0.12 * h))
    top = img_f[:band_h]
    lum = 0.299 * top[:, :, 2] + 0.587 * top[:, :, 1] + 0.114 * top[:, :, 0]
    thr = np.quantile(lum, 0.9)
    mask = lum >= thr
    a = top.mean(axis=(0, 1)) if mask.sum() < 100 else top[mask].mean(axis=0)
    return a.astype(F)


def depth_and_sky(h, w, y_h_ratio=0.42, vx_ratio=0.5, sky_boost=1.25, road_damp=0.9,
                  softness_ratio=0.06):
    """_depth_proxy (fog.py:141-163): (clipped depth, sky weight), f32."""
    yy, xx = np.arange(h, dtype=F), np.arange(w, dtype=F)
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
    return np.clip(d * fac[:, None], F(0), F(1)).astype(F), sw.astype(F)


def depth_bands(depth, beta, depth_blur_max):
    """_depth_blur's per-band kernel sizes (fog.py:194-209): [(band mask,
    rad)] for the bands that blur (rad > 1)."""
    r = np.clip(depth * depth_blur_max * (0.5 + beta), 0.0, depth_blur_max * 1.5)
    out, prev = [], np.zeros_like(depth)
    for b in (0.33, 0.66, 1.0):
        mask = ((depth >= prev) & (depth < b)).astype(F)
        prev = np.full_like(depth, b)
        if mask.sum() < 100:
            continue
        rad = int(max(1, np.mean(r[mask > 0]) * 1.5)) | 1
        if rad <= 1:
            continue
        out.append((mask, rad))
    return out


def glow(img, strength):
    """_glow (fog.py:182-192)."""
    g = gray_u8((img * 255).astype(np.uint8)).astype(F) / 255.0
    thr = np.clip(g.mean() + 0.6 * g.std(), 0.65, 0.9)
    hard = (g > thr).astype(F)
    k = int(9 + 20 * strength) | 1
    soft = np.clip(gaussian_blur(hard, k, k * 0.35), 0, 1)
    k2 = int(max(7, (img.shape[0] + img.shape[1]) * (0.003 + 0.01 * strength))) | 1
    blur = gaussian_blur(img, k2, k2 * 0.25)
    return np.clip(img * (1 - soft[..., None]) + (img + strength * blur) * soft[..., None], 0, 1)


def depth_blur(hazy, depth, strength, depth_blur_max):
    """_depth_blur (fog.py:194-215)."""
    out = hazy.copy()
    for mask, rad in depth_bands(depth, strength, depth_blur_max):
        blurred = gaussian_blur(hazy, rad, rad * 0.5)
        m3 = gaussian_blur(mask, rad | 1, rad * 0.5)[..., None]
        out = out * (1 - m3) + blurred * m3
    return np.clip(out, 0, 1)


def contrast_fade(img, amount):
    """_local_contrast_fade (fog.py:217-225), on the C oracle's YCrCb."""
    from oracle import cpu
    ycc = cpu.bgr2ycrcb((img * 255).astype(np.uint8))
    y = ycc[..., 0]
    d = int(5 + amount * 20) | 1
    ys = bilateral_u8(y, d, 25 + amount * 50, 25 + amount * 50)
    ycc = ycc.copy()
    ycc[..., 0] = add_weighted_u8(y, 1.0 - amount, ys, amount)
    return cpu.ycrcb2bgr(ycc).astype(F) / 255.0


def draw_full(rng, h, w, level="medium", mor=None, scale_ratio=0.18, n_oct=2, rain=False):
    """One frame's draws for the full synthesize, in fog.py's order
    (245-293), keeping every value (airlight tint, target mean, glow,
    contrast drop, the sensor-noise normals)."""
    if mor is not None and mor > 0:
        beta = 3.912 / float(mor)
        a_r, glow_r, cd_r = (0.86, 0.98), (0.12, 0.45), (0.08, 0.22)
    else:
        beta_r, a_r, glow_r, cd_r = PRESETS[level]
        beta = beta_r[0] + (beta_r[1] - beta_r[0]) * rng.rand()
    octs, _ = octaves(h, w, scale_ratio, n_oct)
    g = np.random.RandomState(rng.randint(1e9))
    grids = [g.rand(gh + 1, gw + 1).astype(F) for gh, gw, _ in octs]
    tint_a = rng.uniform(-0.02, 0.02, size=3).astype(F)
    a_target = a_r[0] + (a_r[1] - a_r[0]) * rng.rand()
    glow_s = glow_r[0] + (glow_r[1] - glow_r[0]) * rng.rand()
    cdrop = cd_r[0] + (cd_r[1] - cd_r[0]) * rng.rand()
    tint = (1.0 + rng.uniform(-0.015, 0.02, size=3)).astype(F)
    gamma = 1.0 + rng.uniform(-0.04, 0.05) if rng.rand() < 0.35 else 1.0
    noise = rng.normal(0, 0.0035, size=(h, w, 3)).astype(F) if rng.rand() < 0.3 else None
    seed = rng.randint(1 << 24) if rain else 0
    return dict(beta=beta, grids=grids, tint_a=tint_a, a_target=a_target, glow=glow_s,
                cdrop=cdrop, tint=tint, gamma=gamma, noise=noise, rain_seed=int(seed))


def fog_frame_full(img, prm, y_h_ratio=0.42, vx_ratio=0.5, sky_boost=1.25, road_damp=0.9,
                   softness_ratio=0.06, global_veil=0.06, depth_blur_max=3.5,
                   edge_guided=True, scale_ratio=0.18, n_oct=2, rain_p=0.0, rain_len=16):
    """EnhancedFogSynthesizer.synthesize (fog.py:227-299) with every filter,
    on one (h, w, 3) u8 BGR frame and the draws of draw_full()."""
    h, w = img.shape[:2]
    x = img.astype(F) / 255.0
    depth, sw = depth_and_sky(h, w, y_h_ratio, vx_ratio, sky_boost, road_damp, softness_ratio)
    octs, norm = octaves(h, w, scale_ratio, n_oct)
    nz = noise(h, w, prm["grids"], octs, norm)
    nn = (nz - nz.min()) / max(F(1e-6), nz.max() - nz.min())
    beta_map = (prm["beta"] * (F(0.85) + F(0.35) * nn)).astype(F)
    # airlight (fog.py:120-139, 257-258)
    a_rgb = np.clip(airlight_rgb(x) + prm["tint_a"], 0.7, 1.0)
    vg = np.linspace(1.0, 0.85, h, dtype=F)[:, None, None]
    xg = np.linspace(0.95, 1.05, w, dtype=F)[None, :, None]
    amap = vg * a_rgb[None, None, :] * xg
    for c in range(3):
        amap[:, :, c] = bilateral_f32(amap[:, :, c], 33, 12, 12)
    amap = np.clip(amap, 0.7, 1.0)
    scale = prm["a_target"] / max(1e-6, amap.mean())
    amap = np.clip(amap * scale, 0.75, 1.0)
    # transmission (fog.py:172-179)
    t = np.clip(np.exp(-beta_map * depth), 0.05, 1.0)
    if edge_guided:
        t = np.clip(bilateral_f32(t, 17, 12, 12), 0.05, 1.0)
    t3 = t[..., None]
    hazy = x * t3 + amap * (1.0 - t3)
    gv = (global_veil * (0.6 + 0.4 * sw))[:, None, None]
    hazy = np.clip(hazy * (1.0 - gv) + amap * gv, 0, 1)
    hazy = glow(hazy, prm["glow"])
    hazy = depth_blur(hazy, depth, prm["beta"], depth_blur_max)
    hazy = contrast_fade(hazy, prm["cdrop"])
    hazy = np.clip(hazy * prm["tint"][None, None, :], 0, 1)
    if prm["gamma"] != 1.0:
        hazy = np.clip(hazy ** prm["gamma"], 0, 1)
    if prm["noise"] is not None:
        hazy = np.clip(hazy + prm["noise"], 0, 1)
    if rain_p > 0:
        thr = np.uint32(min(float(np.float32(rain_p)) * 4294967296.0, 4294967295.0))
        yi, xi = np.arange(h)[:, None], np.arange(w)[None, :]
        col = (xi + (yi >> 2)).astype(np.uint32)
        seg = np.broadcast_to((yi // int(rain_len)).astype(np.uint32), col.shape)
        hsh = _lowbias32(np.uint32(prm["rain_seed"]) ^
                         _lowbias32(col * np.uint32(0x9E3779B1) + _lowbias32(seg)))
        rain = (hsh < thr)[..., None]
        hazy = np.where(rain, hazy + (F(1) - hazy) * F(0.45), hazy)
    return (hazy * 255.0 + 0.5).astype(np.uint8)
