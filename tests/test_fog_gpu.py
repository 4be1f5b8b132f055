"""rv_fog_rain_u8 (csrc/augment.hip) vs the CPU oracle (oracle/fog_ref.py).

Tolerance: u8 |d| <= 1 everywhere (the device expf / powf and numpy's differ
by an ulp now and then, which can flip a rounding), and >= 99 % of channel
values exact.  Both sides take the same drawn parameters; the draw itself is
checked bit-for-bit on the CPU (tests/test_fog.py).
"""
import numpy as np
import pytest
import torch

from conftest import road_frame
from oracle import fog_ref

pytestmark = pytest.mark.gpu


def _check(got, ref):
    d = np.abs(got.astype(np.int16) - ref.astype(np.int16))
    exact = float((d == 0).mean())
    assert d.max() <= 1, f"max |d| {d.max()}"
    assert exact >= 0.99, f"exact fraction {exact:.4f}"
    return exact


@pytest.mark.parametrize("H,W,B", [(135, 240, 3), (360, 640, 2), (37, 91, 2), (1280, 1280, 1)])
@pytest.mark.parametrize("kw", [dict(), dict(level="heavy", rain_p=0.004),
                                dict(mor=80.0, perlin_octaves=3)])
def test_fog_matches_oracle(cuda, H, W, B, kw):
    from rvs_amd.augment import FogSynthesizer
    syn = FogSynthesizer(seed=11, device=cuda, filters=False, **kw)
    frames = np.stack([road_frame(H, W, seed=50 + b) for b in range(B)])
    out = syn.synthesize_batch(torch.from_numpy(frames).to(cuda)).cpu().numpy()
    rng = np.random.RandomState(11)
    for b in range(B):
        prm = fog_ref.draw(rng, H, W, level=kw.get("level", "medium"), mor=kw.get("mor"),
                           n_oct=kw.get("perlin_octaves", 2), rain=kw.get("rain_p", 0) > 0)
        ref = fog_ref.fog_frame(frames[b], prm, n_oct=kw.get("perlin_octaves", 2),
                                rain_p=kw.get("rain_p", 0.0))
        _check(out[b], ref)
    assert not np.array_equal(out[0], frames[0])


def test_fog_single_frame_api_and_batch_consistency(cuda):
    from rvs_amd.augment import FogSynthesizer
    H, W = 200, 320
    img = road_frame(H, W, seed=9)
    syn = FogSynthesizer(seed=4, device=cuda, filters=False)
    hazy, meta = syn.synthesize(img)  # numpy in -> numpy out (fog.py:239)
    assert isinstance(hazy, np.ndarray) and hazy.shape == img.shape and hazy.dtype == np.uint8
    assert 0.06 <= meta["beta"] <= 0.12 and meta["y_h"] == int(0.42 * H)
    # the same draw applied inside a batch gives the same bytes
    x = torch.from_numpy(np.stack([img, img[::-1].copy()])).to(cuda)
    draws = [syn.last_draws[0], syn.draw(H, W)]
    out = syn.synthesize_batch(x, draws=draws).cpu().numpy()
    np.testing.assert_array_equal(out[0], hazy)


# --- full synthesize: rv_fog_full_u8 vs oracle.fog_ref.fog_frame_full ---
# The oracle restates every stage in numpy f32 (the OpenCV filters from their
# 4.x scalar forms).  The device differs from it by rounding only: f64 sums
# for the airlight / gray means (numpy: f32), hardware exp in the bilateral's
# colour weight (numpy: the 4096-bin LUT), the airlight map's filter from the
# rank-1 form (< 1e-5), and two truncations to u8 on the way (the glow's
# gray plane and the contrast fade's YCrCb) that turn an ulp into a step.
# Bar: |d| <= 2 and >= 99.9 % of channel values exact (measured r02: all
# frames exact but one, 2e-5 of its values off by 2).

def _check_full(got, ref):
    d = np.abs(got.astype(np.int16) - ref.astype(np.int16))
    exact = float((d == 0).mean())
    print(f"full fog: max |d| {d.max()}, exact {exact:.5f}, |d|>1 {(d > 1).mean():.2e}")
    assert d.max() <= 2, f"max |d| {d.max()}"
    assert exact >= 0.999, f"exact fraction {exact:.4f}"


@pytest.mark.parametrize("H,W,B,kw", [
    (96, 160, 2, dict()),
    (135, 240, 2, dict(level="heavy", rain_p=0.004)),
    (128, 128, 3, dict(mor=80.0, global_veil=0.5, depth_blur_max=4.0, horizon_softness=0.07)),
    (120, 200, 2, dict(level="light", edge_guided=False)),
])
def test_full_fog_matches_oracle(cuda, H, W, B, kw):
    from rvs_amd.augment import FogSynthesizer
    syn = FogSynthesizer(seed=21, device=cuda, **kw)
    frames = np.stack([road_frame(H, W, seed=80 + b) for b in range(B)])
    out = syn.synthesize_batch(torch.from_numpy(frames).to(cuda)).cpu().numpy()
    rng = np.random.RandomState(21)
    opt = {k: kw[k] for k in ("global_veil", "depth_blur_max", "edge_guided") if k in kw}
    if "horizon_softness" in kw:
        opt["softness_ratio"] = kw["horizon_softness"]
    for b in range(B):
        prm = fog_ref.draw_full(rng, H, W, level=kw.get("level", "medium"), mor=kw.get("mor"),
                                rain=kw.get("rain_p", 0) > 0)
        ref = fog_ref.fog_frame_full(frames[b], prm, rain_p=kw.get("rain_p", 0.0), **opt)
        _check_full(out[b], ref)
    assert not np.array_equal(out[0], frames[0])


def test_full_fog_batch_invariance_1280(cuda):
    """config-5 geometry (1280 x 1280): a frame fogged inside a batch of 4 is
    bit-identical to the same frame and draw alone, and the output is a
    plausible haze (brighter, lower contrast than the clean frame)."""
    from rvs_amd.augment import FogSynthesizer
    H = W = 1280
    syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=cuda, global_veil=0.5,
                         depth_blur_max=4.0, horizon_softness=0.07)
    clean = torch.from_numpy(np.stack([road_frame(H, W, seed=70 + b) for b in range(4)])).to(cuda)
    draws = [syn.draw(H, W) for _ in range(4)]
    out = syn.synthesize_batch(clean, draws=draws)
    one = syn.synthesize_batch(clean[2:3].contiguous(), draws=[draws[2]])
    assert torch.equal(out[2], one[0])
    o, c = out.float(), clean.float()
    assert o.mean() > c.mean() and o.std() < c.std()
