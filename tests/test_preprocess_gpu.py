"""Preprocess HIP kernels vs the CPU oracle: bit-exact (uint8 work)."""
import numpy as np
import pytest

from conftest import road_frame
from oracle import cpu

pytestmark = pytest.mark.gpu

SHAPES = [(640, 640), (1080, 1920), (480, 640), (45, 61), (37, 100), (8, 8), (130, 257)]


def _dev(img, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(img)).to(cuda)


@pytest.mark.parametrize("H,W", SHAPES)
@pytest.mark.parametrize("tiles,clip", [(8, 2.0), (4, 0.0), (3, 40.0)])
def test_clahe_bit_exact(cuda, H, W, tiles, clip):
    from rvs_amd import kernels
    img = road_frame(H, W, seed=H + W + tiles)
    got = kernels.clahe_ycrcb(_dev(img, cuda), tiles, clip).cpu().numpy()
    np.testing.assert_array_equal(got, cpu.clahe_ycrcb(img, tiles, clip))


@pytest.mark.parametrize("H,W", SHAPES)
@pytest.mark.parametrize("k", [3, 5, 7, 9])
def test_median_bit_exact(cuda, H, W, k):
    from rvs_amd import kernels
    img = road_frame(H, W, seed=k * 31 + H)  # 1080p k=9: ~2.5 s on the OpenMP oracle
    got = kernels.median(_dev(img, cuda), k).cpu().numpy()
    np.testing.assert_array_equal(got, cpu.median(img, k))


@pytest.mark.parametrize("H,W", SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_fused_clahe_median_equals_chain(cuda, H, W, k):
    from rvs_amd import kernels
    img = road_frame(H, W, seed=H * 3 + k)
    x = _dev(img, cuda)
    if not kernels.clahe_median_fits(x, 8, k):
        pytest.skip("geometry not eligible for the fused pass")
    fused = kernels.clahe_median(x, 8, 2.0, k).cpu().numpy()
    chain = kernels.median(kernels.clahe_ycrcb(x, 8, 2.0), k).cpu().numpy()
    np.testing.assert_array_equal(fused, chain)
    np.testing.assert_array_equal(fused, cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), k))


def test_batched_frames_and_pitch(cuda):
    import torch
    from rvs_amd import kernels
    B, H, W = 5, 120, 200
    frames = np.stack([road_frame(H, W, seed=s) for s in range(B)])
    x = _dev(frames, cuda)
    out = kernels.clahe_median(x, 8, 2.0, 3).cpu().numpy()
    for b in range(B):
        np.testing.assert_array_equal(out[b], cpu.median(cpu.clahe_ycrcb(frames[b]), 3))
    # a padded row pitch (view into a wider buffer) must give the same result
    wide = torch.zeros((B, H, W + 7, 3), dtype=torch.uint8, device=cuda)
    wide[:, :, :W] = x
    view = wide[:, :, :W]
    out2 = kernels.median(kernels.clahe_ycrcb(view, 8, 2.0), 3).cpu().numpy()
    np.testing.assert_array_equal(out2, out)


@pytest.mark.parametrize("H,W", [(1080, 1920), (640, 640), (480, 640), (720, 1280), (37, 91),
                                 (300, 2000), (700, 500)])
def test_letterbox_bit_exact(cuda, H, W):
    from rvs_amd import kernels
    img = road_frame(H, W, seed=H)
    geo = kernels.letterbox_geometry(H, W)
    got = kernels.letterbox(_dev(img, cuda)[None], geo)[0].cpu().numpy()
    np.testing.assert_array_equal(got, cpu.letterbox(img, geo))


def test_gray_span(cuda):
    from rvs_amd import kernels
    imgs = np.stack([road_frame(64, 96, seed=s) for s in range(3)])
    imgs[1] = 77  # flat frame -> span 0
    span = kernels.gray_span(_dev(imgs, cuda)).cpu().numpy()
    for b in range(3):
        y = cpu.bgr2ycrcb(imgs[b])[..., 0].astype(int)
        assert span[b] == y.max() - y.min()


def test_pipeline_matches_reference_semantics(cuda):
    from rvs_amd.preprocess import PreprocessPipeline
    cfg = {"enabled": True,
           "chain": [{"name": "CLAHEDehaze", "params": {"space": "YCrCb", "clip_limit": 2.0,
                                                         "tile_grid": 8}},
                     {"name": "MedianDerain", "params": {"ksize": 4}}],
           "auto_gate": {"enable_low_contrast_gate": False}}
    p = PreprocessPipeline(cfg)
    img = road_frame(96, 128, seed=9)
    out = p(img)
    assert isinstance(out, np.ndarray)
    # ksize 4 -> 5 (median_derain.py:12)
    np.testing.assert_array_equal(out, cpu.median(cpu.clahe_ycrcb(img), 5))
    # gate on: high-contrast frame is returned unchanged (pipeline.py:37-40)
    cfg["auto_gate"] = {"enable_low_contrast_gate": True, "contrast_thresh": 20.0}
    p2 = PreprocessPipeline(cfg)
    assert p2(img) is img
    flat = np.full((32, 32, 3), 90, np.uint8)
    flat[0, 0] = 95
    np.testing.assert_array_equal(p2(flat), cpu.median(cpu.clahe_ycrcb(flat), 5))
    # batched gate: low-contrast frames run the chain, the others pass through
    # untouched (the chain is only run on the gathered low-contrast frames)
    import torch
    frames = []
    for i in range(5):
        f = road_frame(48, 64, seed=40 + i)
        if i in (1, 3):  # squeeze to a span < 20
            f = (90 + (f.astype(np.int32) - 90) // 16).clip(0, 255).astype(np.uint8)
        frames.append(f)
    batch = np.stack(frames)
    span = [int(cpu_gray_span(f)) for f in frames]
    assert [s < 20 for s in span] == [False, True, False, True, False]
    got = p2(torch.from_numpy(batch).to(cuda)).cpu().numpy()
    for i, f in enumerate(frames):
        want = cpu.median(cpu.clahe_ycrcb(f), 5) if span[i] < 20 else f
        np.testing.assert_array_equal(got[i], want)
    flat_batch = torch.from_numpy(batch[[0, 2]].copy()).to(cuda)
    assert p2(flat_batch) is flat_batch  # no low-contrast frame: input returned


def cpu_gray_span(img):
    """cv2.cvtColor BGR2GRAY (14-bit) max - min (pipeline.py:24-30)."""
    i = img.astype(np.int32)
    g = (i[..., 0] * 1868 + i[..., 1] * 9617 + i[..., 2] * 4899 + 8192) >> 14
    return g.max() - g.min()


def test_median_vector_path_ragged_width(cuda):
    """Row pitch a multiple of 4 with W % 4 != 0: dword loads/stores on the
    interior groups, byte path on the ragged right edge."""
    import torch
    from rvs_amd import kernels
    H, W = 70, 130
    img = road_frame(H, W, seed=5)
    wide = torch.zeros((2, H, W + 2, 3), dtype=torch.uint8, device=cuda)
    wide[:, :, :W] = _dev(img, cuda)
    view = wide[:, :, :W]
    out = kernels.clahe_median(view, 8, 2.0, 3)
    ref = cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), 3)
    for b in range(2):
        np.testing.assert_array_equal(out[b].cpu().numpy(), ref)
    np.testing.assert_array_equal(kernels.median(view, 3)[0].cpu().numpy(), cpu.median(img, 3))


@pytest.mark.parametrize("H,W", [(1080, 1920), (720, 1280), (640, 640), (480, 640), (2160, 3840),
                                 (37, 91), (300, 2000), (700, 500), (1000, 1400)])
def test_fused_letterbox_equals_chain(cuda, H, W):
    """rv_clahe_median_letterbox_u8 == rv_clahe_median_u8 + rv_letterbox_u8
    == oracle (CLAHE -> median -> LetterBox), byte for byte."""
    from rvs_amd import _lib, kernels
    img = road_frame(H, W, seed=H + 2 * W)
    x = _dev(np.stack([img, img[::-1].copy()]), cuda)
    geo = kernels.letterbox_geometry(H, W)
    if not kernels.clahe_median_letterbox_fits(H, W, 8, 3, geo):
        with pytest.raises(_lib.RVError):
            kernels.clahe_median_letterbox(x, 8, 2.0, 3, geo)
        pytest.skip("geometry not eligible for the fused letterbox (checked: RV_EINVAL)")
    proc, lb = kernels.clahe_median_letterbox(x, 8, 2.0, 3, geo)
    chain = kernels.clahe_median(x, 8, 2.0, 3)
    np.testing.assert_array_equal(proc.cpu().numpy(), chain.cpu().numpy())
    np.testing.assert_array_equal(lb.cpu().numpy(), kernels.letterbox(chain, geo).cpu().numpy())
    ref = cpu.letterbox(cpu.median(cpu.clahe_ycrcb(img, 8, 2.0), 3), geo)
    np.testing.assert_array_equal(lb[0].cpu().numpy(), ref)


@pytest.mark.parametrize("H,W,tiles,clip", [(1080, 1920, 8, 2.0), (640, 640, 8, 2.0),
                                            (37, 91, 3, 2.0), (480, 640, 8, 0.0),
                                            (721, 1283, 5, 4.0)])
def test_clahe_lab_bit_exact(cuda, H, W, tiles, clip):
    """CLAHEDehaze space='LAB' (rv_clahe_lab_u8) vs the C oracle, bit-exact."""
    from rvs_amd import kernels
    B = 2
    frames = np.stack([road_frame(H, W, seed=60 + b) for b in range(B)])
    frames[1, : H // 3] = (frames[1, : H // 3].astype(int) * [1, 1, 2] // [1, 1, 1]
                           ).clip(0, 255).astype(np.uint8)  # saturated reds
    got = kernels.clahe_lab(_dev(frames, cuda), tiles, clip).cpu().numpy()
    for b in range(B):
        np.testing.assert_array_equal(got[b], cpu.clahe_lab(frames[b], tiles, clip))


def test_lab_chain_through_pipeline(cuda):
    from rvs_amd.preprocess import PreprocessPipeline
    cfg = {"enabled": True,
           "chain": [{"name": "CLAHEDehaze", "params": {"space": "lab", "clip_limit": 2.0,
                                                         "tile_grid": 8}},
                     {"name": "MedianDerain", "params": {"ksize": 3}}]}
    p = PreprocessPipeline(cfg)
    assert not p._fused  # the fused passes are YCrCb-only
    img = road_frame(360, 640, seed=12)
    out = p(img)
    np.testing.assert_array_equal(out, cpu.median(cpu.clahe_lab(img, 8, 2.0), 3))


@pytest.mark.parametrize("H,W,B", [(1080, 1920, 3), (2, 2, 1), (6, 10, 2), (480, 642, 2)])
def test_nv12_to_bgr_bit_exact(cuda, H, W, B):
    """rv_nv12_to_bgr_u8 vs the C oracle (cv2.COLOR_YUV2BGR_NV12), bit-exact;
    W % 4 != 0 takes the scalar path."""
    import torch
    from rvs_amd import kernels
    rng = np.random.default_rng(H + W)
    nv = rng.integers(0, 256, (B, H * 3 // 2, W), dtype=np.uint8)
    got = kernels.nv12_to_bgr(torch.from_numpy(nv).to(cuda)).cpu().numpy()
    for b in range(B):
        np.testing.assert_array_equal(got[b], cpu.nv12_to_bgr(nv[b, :H], nv[b, H:]))
    one = kernels.nv12_to_bgr(torch.from_numpy(nv[0]).to(cuda)).cpu().numpy()
    np.testing.assert_array_equal(one, got[0])
