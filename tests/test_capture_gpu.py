"""Capture front end on the GPU: frames read by the native reader threads,
uploaded as NV12 and converted on the device equal the C oracle's
cv2.COLOR_YUV2BGR_NV12 of the same bytes, bit for bit; the batched pipeline
(MultiStreamCapture: copy stream, event-polled slot release, one batch of
prefetch) keeps every stream's frames in order and feeds RoadVisionEngine."""
import numpy as np
import pytest
import torch

from conftest import road_frame
from oracle import cpu
from test_capture import _i420_planes

pytestmark = pytest.mark.gpu


def _oracle_bgr(y, u, v):
    uv = np.stack([u, v], axis=-1).reshape(u.shape[0], -1)
    return cpu.nv12_to_bgr(y, uv)


def test_video_source_read_matches_oracle(cuda, tmp_path):
    from rvs_amd.io_video import VideoSource, write_y4m
    p = tmp_path / "cam.y4m"
    write_y4m(str(p), [road_frame(90, 160, seed=s) for s in range(4)])
    planes, W, H = _i420_planes(p)
    src = VideoSource(str(p), device=cuda)
    for y, u, v in planes:
        fr = src.read()
        assert fr.ok and fr.image.shape == (H, W, 3) and fr.ts > 0
        np.testing.assert_array_equal(fr.image, _oracle_bgr(y, u, v))
    assert not src.read().ok
    src.release()


@pytest.mark.parametrize("prefetch", [True, False])
def test_multistream_capture_feeds_engine(cuda, tmp_path, prefetch):
    from rvs_amd.config import load_config
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.io_video import MultiStreamCapture, write_y4m
    S, F, H, W = 4, 5, 120, 200
    paths = []
    for s in range(S):
        p = tmp_path / f"cam{s}.y4m"
        write_y4m(str(p), [road_frame(H, W, seed=1000 * s + f) for f in range(F)])
        paths.append(str(p))
    planes = [_i420_planes(p)[0] for p in paths]
    cap = MultiStreamCapture(paths, device=cuda, nbuf=3, prefetch=prefetch)
    assert (cap.S, cap.H, cap.W) == (S, H, W)
    cfg = load_config()
    cfg["detect"]["weights"] = "synthetic"
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    last_ts = np.zeros(S)
    for f in range(F):
        got = cap.next_batch()
        assert got is not None
        frames, ts, idx = got
        assert list(idx) == [f] * S
        out = eng.step(frames, ts)
        host = frames.cpu().numpy()
        for s in range(S):
            np.testing.assert_array_equal(host[s], _oracle_bgr(*planes[s][f]))
        t = ts.cpu().numpy()
        assert (t >= last_ts).all()
        last_ts = t
        if f == 0:
            proc = out["proc"].cpu().numpy()
            np.testing.assert_array_equal(proc[1], cpu.median(cpu.clahe_ycrcb(host[1]), 3))
        eng.results(out)
    assert cap.next_batch() is None
    cap.close()
    eng.close()
