"""Integration: the batched engine (preprocess -> detect -> track) on a few
streams, checked stage by stage against the oracle fed with the GPU's own
upstream outputs: proc frames bit-exact; NMS exact on the GPU's raw
prediction; SORT ids/distances exact on the GPU's detections."""
import numpy as np
import pytest
import torch

from oracle import cpu, sort_ref, yolo_ref

pytestmark = pytest.mark.gpu

IMG = [[560, 1000], [1360, 1000], [1160, 620], [760, 620]]
WLD = [[-3.5, 5.0], [3.5, 5.0], [3.5, 30.0], [-3.5, 30.0]]


def test_engine_steps_match_oracle(cuda):
    from rvs_amd.config import load_config
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = load_config()
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = IMG
    cfg["geometry"]["projector"]["world_points"] = WLD
    S, H, W, F = 3, 1080, 1920, 6
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    frames = road_frames(S, F, H, W, device=cuda)
    oproj = sort_ref.HomographyProjector(eng.projector._H, (0.0, 0.0), 1000.0)
    trackers = [sort_ref.SortTracker(cfg["tracking"]) for _ in range(S)]
    raw = torch.empty((S, 84, eng.detector.A), dtype=torch.float32, device=cuda)
    for f in range(F):
        ts = torch.full((S,), f / 30.0, dtype=torch.float64, device=cuda)
        out = eng.step(frames[f], ts)
        res = eng.results(out)
        proc = out["proc"].cpu().numpy()
        src = frames[f].cpu().numpy()
        for s in range(S):
            np.testing.assert_array_equal(proc[s], cpu.median(cpu.clahe_ycrcb(src[s]), 3))
        # NMS on the GPU's own raw prediction (same proc frames)
        eng.detector.forward_raw(eng.detector.letterbox(out["proc"]), raw, candidates=False)
        ref = yolo_ref.postprocess(raw.cpu().numpy(), (eng.detector.in_h, eng.detector.in_w),
                                   (H, W), classes_keep=cfg["detect"]["classes_keep"])
        for s in range(S):
            got = np.array([[d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id] for d in res[s]],
                           np.float32).reshape(-1, 6)
            np.testing.assert_array_equal(got, ref[s])
            dets = [sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in ref[s]]
            trackers[s].update(dets, f / 30.0, oproj)
            assert [d.track_id for d in res[s]] == [d.track_id for d in dets]
            assert [d.distance_m for d in res[s]] == [d.distance_m for d in dets]
    eng.close()


@pytest.mark.parametrize("depth,chunk", [(2, None), (3, 1), (3, 3), (3, None), (3, 0)])
def test_overlapped_steps_match_sequential_steps(cuda, depth, chunk):
    """bench.py's timed mode (engine.OverlappedSteps): the track stage of step
    k runs on a side stream beside the preprocess of step k+1, with `chunk`
    pipeline stages per captured graph (None = the default 8, 0 = one graph).
    The final detections, track ids, proc frames and the whole SORT state must
    equal those of plain sequential step() calls."""
    from rvs_amd.config import load_config
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = load_config()
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = IMG
    cfg["geometry"]["projector"]["world_points"] = WLD
    S, H, W, F = 4, 1080, 1920, 6
    frames = road_frames(S, F, H, W, device=cuda)
    ts = torch.tensor([[f / 30.0] * S for f in range(F)], dtype=torch.float64, device=cuda)
    seq = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    for f in range(F):
        out_seq = seq.step(frames[f], ts[f])
    ovl = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    ovl.step(frames[0], ts[0])  # eager first step (one-time kernel setup)
    run = OverlappedSteps(ovl, [frames[f] for f in range(1, F)], [ts[f] for f in range(1, F)],
                          depth=depth, chunk=chunk)
    run.run()
    torch.cuda.synchronize()
    r_seq, r_ovl = seq.results(out_seq), ovl.results(run.outs[-1])
    key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id, d.distance_m,  # noqa
                       d.speed_kmh) for d in s] for s in r]
    assert key(r_seq) == key(r_ovl)
    np.testing.assert_array_equal(run.outs[-1]["proc"].cpu().numpy(), out_seq["proc"].cpu().numpy())
    Ts, xs, ms = seq.tracker.export()
    To, xo, mo = ovl.tracker.export()
    np.testing.assert_array_equal(Ts, To)
    for s in range(S):
        np.testing.assert_array_equal(xs[s, :Ts[s]], xo[s, :To[s]])
        np.testing.assert_array_equal(ms[s, :Ts[s]], mo[s, :To[s]])
    seq.close()
    ovl.close()
