"""Pin the C oracle's preprocess restatements (CPU only).

OpenCV is absent from this container, so CLAHE / colour /
median parity against real OpenCV is UNPINNED.  What is pinned here:
  * colour conversion: hand-derived known answers;
  * median: scipy.ndimage.median_filter(mode='nearest') -- an independent
    exact-median implementation with cv2.medianBlur's replicate border;
  * CLAHE: a second, independent numpy restatement (float32 scalar semantics)
    written from the published algorithm, on small frames;
  * letterbox: exact 3x decimation at 1080p (integral source coordinates).
"""
import numpy as np
import pytest
import scipy.ndimage

from conftest import road_frame
from oracle import cpu


def test_ycrcb_known_answers():
    px = np.array([[[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 0, 255], [10, 200, 30]]],
                  np.uint8)
    ycc = cpu.bgr2ycrcb(px)
    # Y = (B*1868 + G*9617 + R*4899 + 8192) >> 14
    assert ycc[0, 0].tolist() == [0, 128, 128]
    assert ycc[0, 1].tolist() == [255, 128, 128]
    yb = (255 * 1868 + 8192) >> 14
    assert ycc[0, 2, 0] == yb
    assert ycc[0, 2, 2] == min(255, ((255 - yb) * 9241 + (128 << 14) + 8192) >> 14)
    yr = (255 * 4899 + 8192) >> 14
    assert ycc[0, 3, 1] == min(255, ((255 - yr) * 11682 + (128 << 14) + 8192) >> 14)
    back = cpu.ycrcb2bgr(ycc)
    assert np.abs(back.astype(int) - px.astype(int)).max() <= 2


@pytest.mark.parametrize("k", [3, 5, 7, 9])
@pytest.mark.parametrize("shape", [(17, 23), (64, 48), (5, 5), (1, 7)])
def test_median_matches_scipy(k, shape):
    rng = np.random.default_rng(k * 100 + shape[0])
    img = rng.integers(0, 256, size=shape + (3,), dtype=np.uint8)
    ref = scipy.ndimage.median_filter(img, size=(k, k, 1), mode="nearest")
    np.testing.assert_array_equal(cpu.median(img, k), ref)


def _clahe_numpy(plane, tiles, clip):
    """Independent numpy restatement of cv::CLAHE (8UC1)."""
    H, W = plane.shape
    if W % tiles == 0 and H % tiles == 0:
        tw, th = W // tiles, H // tiles
        ext = plane
    else:
        ext = np.pad(plane, ((0, tiles - H % tiles), (0, tiles - W % tiles)), mode="reflect")
        th, tw = ext.shape[0] // tiles, ext.shape[1] // tiles
    area = tw * th
    clip_limit = 0
    if clip > 0:
        clip_limit = max(int(clip * area / 256), 1)
    lut_scale = np.float32(255) / np.float32(area)
    lut = np.zeros((tiles, tiles, 256), np.uint8)
    for ty in range(tiles):
        for tx in range(tiles):
            t = ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
            h = np.bincount(t.ravel(), minlength=256).astype(np.int64)
            if clip_limit > 0:
                clipped = int(np.maximum(h - clip_limit, 0).sum())
                h = np.minimum(h, clip_limit)
                h += clipped // 256
                residual = clipped % 256
                if residual:
                    step = max(256 // residual, 1)
                    idx = np.arange(0, 256, step)[:residual]
                    h[idx] += 1
            s = np.cumsum(h).astype(np.float32) * lut_scale
            lut[ty, tx] = np.clip(np.rint(s), 0, 255).astype(np.uint8)
    inv_tw = np.float32(1.0) / np.float32(tw)
    inv_th = np.float32(1.0) / np.float32(th)
    xs = np.arange(W, dtype=np.float32) * inv_tw - np.float32(0.5)
    ys = np.arange(H, dtype=np.float32) * inv_th - np.float32(0.5)
    tx1 = np.floor(xs).astype(int)
    xa = (xs - tx1.astype(np.float32)).astype(np.float32)
    xa1 = (np.float32(1) - xa).astype(np.float32)
    ty1 = np.floor(ys).astype(int)
    ya = (ys - ty1.astype(np.float32)).astype(np.float32)
    ya1 = (np.float32(1) - ya).astype(np.float32)
    tx2 = np.minimum(tx1 + 1, tiles - 1)
    tx1 = np.maximum(tx1, 0)
    ty2 = np.minimum(ty1 + 1, tiles - 1)
    ty1 = np.maximum(ty1, 0)
    out = np.zeros_like(plane)
    for y in range(H):
        v = plane[y].astype(int)
        l11 = lut[ty1[y], tx1, v].astype(np.float32)
        l12 = lut[ty1[y], tx2, v].astype(np.float32)
        l21 = lut[ty2[y], tx1, v].astype(np.float32)
        l22 = lut[ty2[y], tx2, v].astype(np.float32)
        res = (l11 * xa1 + l12 * xa) * ya1[y] + (l21 * xa1 + l22 * xa) * ya[y]
        out[y] = np.clip(np.rint(res.astype(np.float32)), 0, 255).astype(np.uint8)
    return out


@pytest.mark.parametrize("H,W,tiles,clip", [(64, 64, 8, 2.0), (48, 80, 8, 2.0), (45, 61, 8, 2.0),
                                            (40, 40, 4, 0.0), (33, 64, 2, 4.0),
                                            (64, 48, 8, 40.0)])
def test_clahe_c_oracle_matches_numpy_restatement(H, W, tiles, clip):
    img = road_frame(H, W, seed=H * 7 + W)
    plane = cpu.bgr2ycrcb(img)[..., 0].copy()
    np.testing.assert_array_equal(cpu.clahe_u8c1(plane, tiles, clip),
                                  _clahe_numpy(plane, tiles, clip))


def test_clahe_constant_plane_known_answer():
    # constant plane: one bin holds the whole tile; after clipping, the LUT
    # at that value is round(255/area * (cdf)).  Every pixel blends 4 equal
    # LUT entries, so the output is that entry.
    plane = np.full((16, 16), 100, np.uint8)
    out = cpu.clahe_u8c1(plane, 2, 2.0)
    area = 64
    clip_limit = max(int(2.0 * area / 256), 1)  # 1
    clipped = area - clip_limit
    h = np.zeros(256, int)
    h[100] = clip_limit
    h += clipped // 256
    res = clipped % 256
    step = max(256 // res, 1)
    h[np.arange(0, 256, step)[:res]] += 1
    expect = int(np.rint(np.float32(np.cumsum(h)[100]) * (np.float32(255) / np.float32(area))))
    assert (out == expect).all()


def test_letterbox_1080p_is_exact_decimation():
    img = road_frame(1080, 1920, seed=3)
    geo = cpu.letterbox_geometry(1080, 1920)
    lb = cpu.letterbox(img, geo)
    assert lb.shape == (384, 640, 3)
    assert (lb[:12] == 114).all() and (lb[-12:] == 114).all()
    np.testing.assert_array_equal(lb[12:372], img[1::3, 1::3])


def test_letterbox_identity_at_640():
    img = road_frame(640, 640, seed=4)
    geo = cpu.letterbox_geometry(640, 640)
    np.testing.assert_array_equal(cpu.letterbox(img, geo), img)


# --- LAB path (clahe_dehaze.py:21-25) ------------------------------------
def _cie_lab8(bgr):
    """Float CIE L*a*b* (sRGB, D65) scaled to OpenCV's 8U ranges."""
    c = bgr[..., ::-1].astype(np.float64) / 255.0
    lin = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
    m = np.array([[0.412453, 0.357580, 0.180423], [0.212671, 0.715160, 0.072169],
                  [0.019334, 0.119193, 0.950227]])
    xyz = lin @ m.T / np.array([0.950456, 1.0, 1.088754])
    f = np.where(xyz > 216 / 24389, np.cbrt(xyz), xyz * 841 / 108 + 16 / 116)
    L = 116 * f[..., 1] - 16
    a = 500 * (f[..., 0] - f[..., 1])
    b = 200 * (f[..., 1] - f[..., 2])
    return np.stack([L * 255 / 100, a + 128, b + 128], -1)


def test_lab_known_answers():
    px = np.array([[[255, 255, 255], [0, 0, 0], [128, 128, 128], [0, 0, 255], [0, 255, 0],
                    [255, 0, 0]]], np.uint8)
    lab = cpu.bgr2lab(px)
    assert lab[0, 0].tolist() == [255, 128, 128] and lab[0, 1].tolist() == [0, 128, 128]
    # CIE values: red (53.24, 80.09, 67.20), green (87.73, -86.18, 83.18),
    # blue (32.30, 79.19, -107.86), gray 128 (53.59, 0, 0)
    assert lab[0, 2].tolist() == [137, 128, 128]
    assert lab[0, 3].tolist() == [136, 208, 195]
    assert lab[0, 4].tolist() == [224, 42, 211]
    assert lab[0, 5].tolist() == [82, 207, 20]
    back = cpu.lab2bgr(lab)
    assert back[0, 0].tolist() == [255, 255, 255] and back[0, 1].tolist() == [0, 0, 0]
    assert back[0, 2].tolist() == [128, 128, 128]


def test_lab_matches_cie_float():
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (1, 50000, 3), dtype=np.uint8)
    d = np.abs(cpu.bgr2lab(x).astype(np.float64) - _cie_lab8(x))
    # the 11-bit linear-light table quantises dark colours: measured max 2.1
    # LSB (a channel), > 1 LSB for 0.3 % of values
    assert d.max() <= 2.5 and (d > 1.0).mean() < 0.01, d.max()
    # the inverse recovers grays within 1 LSB (L has 256 levels over 0..100)
    # and colours within the 8U Lab quantisation (measured max 22 on
    # saturated colours, mean < 1)
    g = np.repeat(np.arange(256, dtype=np.uint8)[None, :, None], 3, 2)
    rg = cpu.lab2bgr(cpu.bgr2lab(g)).astype(int)
    assert np.abs(rg - g).max() <= 1
    rt = np.abs(cpu.lab2bgr(cpu.bgr2lab(x)).astype(int) - x)
    assert rt.mean() < 1.0 and rt.max() <= 24


def test_lab_tables_in_library_match_oracle():
    import ctypes
    from rvs_amd import _lib
    buf = ctypes.create_string_buffer(cpu.LAB_TABLE_BYTES)
    assert _lib.load().rv_lab_tables_host(buf, cpu.LAB_TABLE_BYTES) == 0
    assert buf.raw == cpu.lab_tables()
    assert _lib.load().rv_lab_tables_host(buf, 100) == -1000


def test_clahe_lab_oracle_structure():
    img = road_frame(120, 160, seed=4)
    out = cpu.clahe_lab(img, 8, 2.0)
    lab_in, lab_out = cpu.bgr2lab(img), cpu.bgr2lab(out)
    # CLAHE equalises L: the L spread grows on a low-contrast road frame
    spread = lambda p: np.percentile(p, 95) - np.percentile(p, 5)  # noqa: E731
    assert spread(lab_out[..., 0]) > spread(lab_in[..., 0])
    # the L plane CLAHE'd by the oracle is exactly what the chain applies
    l2 = cpu.clahe_u8c1(np.ascontiguousarray(lab_in[..., 0]), 8, 2.0)
    merged = lab_in.copy()
    merged[..., 0] = l2
    np.testing.assert_array_equal(out, cpu.lab2bgr(merged))


# --- NV12 ingest (cv2.COLOR_YUV2BGR_NV12) ----------------------------------
def test_nv12_known_answers():
    uv = np.array([[128, 128]], np.uint8)
    assert cpu.nv12_to_bgr(np.full((2, 2), 16, np.uint8), uv)[0, 0].tolist() == [0, 0, 0]
    assert cpu.nv12_to_bgr(np.full((2, 2), 235, np.uint8), uv)[0, 0].tolist() == [255, 255, 255]
    # BT.601 video-range primaries (Y, U, V) -> BGR
    red = cpu.nv12_to_bgr(np.full((2, 2), 81, np.uint8), np.array([[90, 240]], np.uint8))
    blue = cpu.nv12_to_bgr(np.full((2, 2), 41, np.uint8), np.array([[240, 110]], np.uint8))
    assert red[0, 0].tolist() == [0, 0, 254] and blue[0, 0].tolist() == [255, 0, 0]


def test_nv12_matches_bt601_float():
    rng = np.random.default_rng(5)
    H, W = 64, 96
    y = rng.integers(0, 256, (H, W), dtype=np.uint8)
    uv = rng.integers(0, 256, (H // 2, W), dtype=np.uint8)
    got = cpu.nv12_to_bgr(y, uv).astype(np.float64)
    u = np.repeat(np.repeat(uv[:, 0::2].astype(np.float64) - 128, 2, 0), 2, 1)
    v = np.repeat(np.repeat(uv[:, 1::2].astype(np.float64) - 128, 2, 0), 2, 1)
    yy = 1.164 * np.maximum(y.astype(np.float64) - 16, 0)
    ref = np.stack([yy + 2.018 * u, yy - 0.391 * u - 0.813 * v, yy + 1.596 * v], -1)
    d = np.abs(got - np.clip(ref, 0, 255))
    assert d.max() <= 1.5  # fixed-point truncation vs the rounded float matrix


def test_nv12_abi_argument_errors():
    import ctypes
    from rvs_amd import _lib
    lib = _lib.load()
    p = ctypes.c_void_p(64)
    assert lib.rv_nv12_to_bgr_u8(None, p, 4, 4, 24, 8, p, 1, 4, 4, 12, None) == -1000
    assert lib.rv_nv12_to_bgr_u8(p, p, 4, 4, 24, 8, p, 1, 3, 4, 12, None) == -1000  # odd H
    assert lib.rv_nv12_to_bgr_u8(p, p, 4, 4, 8, 8, p, 1, 4, 4, 12, None) == -1000  # stride
    assert lib.rv_nv12_to_bgr_u8(p, p, 4, 4, 24, 8, p, 0, 4, 4, 12, None) == 0  # B = 0
