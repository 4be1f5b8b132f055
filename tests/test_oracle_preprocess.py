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
