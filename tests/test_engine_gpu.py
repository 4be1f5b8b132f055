"""Integration: the batched engine (preprocess -> detect -> track -> hand-back)
checked stage by stage against the oracle fed with the GPU's own upstream
outputs: proc frames bit-exact; NMS exact on the GPU's raw prediction (the
same kernel sequence as the candidate path); SORT ids / distances exact and
speeds to 1e-9 relative on the GPU's detections; no stream overflows tmax.

test_bench_configuration_parity runs exactly what bench.py times: 32
streams of 1080p, per-layer autotuned conv kernels, the 3-deep software
pipeline of 8 steps per captured graph, results handed back to pinned host
records inside the step (reference call order: main_preview.py:94-109)."""
import numpy as np
import pytest
import torch

from oracle import cpu, sort_ref, yolo_ref

pytestmark = pytest.mark.gpu

IMG = [[560, 1000], [1360, 1000], [1160, 620], [760, 620]]
WLD = [[-3.5, 5.0], [3.5, 5.0], [3.5, 30.0], [-3.5, 30.0]]


def _cfg():
    from rvs_amd.config import load_config
    cfg = load_config()
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = IMG
    cfg["geometry"]["projector"]["world_points"] = WLD
    return cfg


class Checker:
    """Per-stream oracle state: the reference-semantics SORT (sort_ref) fed
    with the oracle NMS of the GPU's own raw prediction."""

    def __init__(self, eng, cfg, proc_streams):
        self.eng, self.cfg = eng, cfg
        self.S = eng.S
        self.proj = sort_ref.HomographyProjector(eng.projector._H, (0.0, 0.0), 1000.0)
        self.trackers = [sort_ref.SortTracker(cfg["tracking"]) for _ in range(self.S)]
        self.proc_streams = proc_streams
        self.raw = torch.empty((self.S, 84, eng.detector.A), dtype=torch.float32,
                               device=eng.device)
        self.n_dets = 0

    def check(self, frames, proc, res, t):
        eng, S = self.eng, self.S
        src = frames.cpu().numpy()
        pr = proc.cpu().numpy()
        for s in self.proc_streams:
            np.testing.assert_array_equal(pr[s], cpu.median(cpu.clahe_ycrcb(src[s]), 3))
        # the production kernel sequence (fused stem, tuned configs) with the
        # raw prediction also written out
        eng.detector.set_raw_fused(True)
        eng.detector.forward_raw(eng.detector.letterbox(proc), self.raw, candidates=False)
        eng.detector.set_raw_fused(False)
        ref = yolo_ref.postprocess(self.raw.cpu().numpy(), (eng.detector.in_h, eng.detector.in_w),
                                   (eng.H, eng.W), classes_keep=self.cfg["detect"]["classes_keep"])
        for s in range(S):
            got = np.array([[d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id] for d in res[s]],
                           np.float32).reshape(-1, 6)
            np.testing.assert_array_equal(got, ref[s])
            dets = [sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in ref[s]]
            self.trackers[s].update(dets, t, self.proj)
            assert [d.track_id for d in res[s]] == [d.track_id for d in dets]
            assert [d.distance_m for d in res[s]] == [d.distance_m for d in dets]
            for a, b in zip(res[s], dets):
                assert (a.speed_kmh is None) == (b.speed_kmh is None)
                if a.speed_kmh is not None:
                    assert abs(a.speed_kmh - b.speed_kmh) <= 1e-9 * max(1.0, abs(b.speed_kmh))
            self.n_dets += len(dets)


def test_engine_steps_match_oracle(cuda):
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W, F = 3, 1080, 1920, 6
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    frames = road_frames(S, F, H, W, device=cuda)
    chk = Checker(eng, cfg, range(S))
    for f in range(F):
        ts = torch.full((S,), f / 30.0, dtype=torch.float64, device=cuda)
        out = eng.step(frames[f], ts)
        res = eng.results(out)
        chk.check(frames[f], out["proc"], res, f / 30.0)
    st = eng.track_stats()
    assert st["overflow"].sum() == 0
    np.testing.assert_array_equal(st["T"], [len(t.tracks) for t in chk.trackers])
    eng.close()


def test_results_record_matches_device_outputs(cuda):
    """The hand-back record (rv_results_handback) equals the device tensors
    it was packed from (the reference's .cpu().numpy() hand-over)."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W = 4, 1080, 1920
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    frames = road_frames(S, 3, H, W, device=cuda)
    for f in range(3):
        out = eng.step(frames[f], torch.full((S,), f / 30.0, dtype=torch.float64, device=cuda))
    a = eng.results(out)
    b = eng.results({k: v for k, v in out.items() if k != "record"})
    key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.cls_name, d.track_id,  # noqa
                       d.distance_m, d.speed_kmh) for d in s] for s in r]
    assert key(a) == key(b)
    assert sum(len(s) for s in a) > 0
    eng.close()


@pytest.mark.parametrize("depth,chunk,lanes,pair", [
    (2, None, 1, 1), (3, 1, 1, 1), (3, 3, 1, 1), (3, None, 1, 1), (3, 0, 1, 1), (3, None, 2, 1),
    (3, 3, 2, 1), (3, 0, 3, 1), (4, None, 2, 1), (4, 3, 2, 1), (4, 0, 2, 1), (4, None, 2, 2),
    (4, 1, 2, 2)])
def test_overlapped_steps_match_sequential_steps(cuda, depth, chunk, lanes, pair):
    """bench.py's timed mode (engine.OverlappedSteps): the track stage of step
    k runs on a side stream beside the preprocess of step k+1, with `chunk`
    pipeline stages per captured graph (None = the default 8, 0 = one graph);
    lanes >= 2 (depth 3): the dependency-graph schedule with that many concurrent YOLO
    forwards; pair 2 (depth 4): one forward over two consecutive steps'
    frames.  EVERY step's handed-back detections / track ids and proc
    frames, and the final SORT state, must equal those of plain sequential
    step() calls."""
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W = 4, 1080, 1920
    F = 9 if pair == 2 else 8  # the overlapped steps (F - 1) pair up
    frames = road_frames(S, F, H, W, device=cuda)
    ts = torch.tensor([[f / 30.0] * S for f in range(F)], dtype=torch.float64, device=cuda)
    seq = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    seq_res, seq_proc = [], []
    for f in range(F):
        out_seq = seq.step(frames[f], ts[f])
        seq_res.append(seq.results(out_seq))
        seq_proc.append(out_seq["proc"].cpu().numpy())
    ovl = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=lanes, pair=pair)
    ovl.step(frames[0], ts[0])  # eager first step (one-time kernel setup)
    run = OverlappedSteps(ovl, [frames[f] for f in range(1, F)], [ts[f] for f in range(1, F)],
                          depth=depth, chunk=chunk)
    run.run()
    torch.cuda.synchronize()
    key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id, d.distance_m,  # noqa
                       d.speed_kmh) for d in s] for s in r]
    assert len(run.outs) == F - 1
    for k, o in enumerate(run.outs):
        assert key(seq_res[k + 1]) == key(ovl.results(o)), f"step {k + 1}"
        np.testing.assert_array_equal(o["proc"].cpu().numpy(), seq_proc[k + 1])
    Ts, xs, ms = seq.tracker.export()
    To, xo, mo = ovl.tracker.export()
    np.testing.assert_array_equal(Ts, To)
    for s in range(S):
        np.testing.assert_array_equal(xs[s, :Ts[s]], xo[s, :To[s]])
        np.testing.assert_array_equal(ms[s, :Ts[s]], mo[s, :To[s]])
    seq.close()
    ovl.close()


@pytest.mark.parametrize("depth,lanes,pair", [(4, 2, 1), (4, 2, 4), (3, 1, 1)])
def test_bench_configuration_parity(cuda, depth, lanes, pair):
    """Exactly bench.py's timed configuration (S = 32 streams of 1080p,
    autotuned conv kernels, OverlappedSteps(depth=4, chunk=8) on two forward
    lanes, with and without pairing two steps per forward -- and the depth-3
    one-lane pipeline --, hand-back into per-step
    host records), checked against the oracle on every step:
    proc bit-exact on a sample of streams, NMS exact on the GPU's raw
    prediction for all 32 streams, SORT ids / distances exact for all 32
    streams, and no stream ever exceeds tmax."""
    from rvs_amd.engine import OverlappedSteps, RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W, WARM, K = 32, 1080, 1920, 2, 8
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=lanes, pair=pair)
    frames = road_frames(S, WARM + K, H, W, device=cuda)
    ts = torch.tensor([[f / 30.0] * S for f in range(WARM + K)], dtype=torch.float64, device=cuda)
    chk = Checker(eng, cfg, proc_streams=[0, 13, 31])
    for f in range(WARM):
        out = eng.step(frames[f], ts[f])
        chk.check(frames[f], out["proc"], eng.results(out), f / 30.0)
    eng.autotune(frames[0], reps=1)
    assert len(eng.detector.tuned_configs()) > 0
    # bench.py's --conv-grid persistent: the tuned tiles on persistent grids
    eng.detector.load_tuned([tuple(c[:4]) + (1,) + tuple(c[5:])
                             for c in eng.detector.tuned_configs()])
    run = OverlappedSteps(eng, [frames[WARM + k] for k in range(K)],
                          [ts[WARM + k] for k in range(K)], depth=depth, chunk=8)
    run.run()
    torch.cuda.synchronize()
    for k, o in enumerate(run.outs):
        chk.check(frames[WARM + k], o["proc"], eng.results(o), (WARM + k) / 30.0)
    st = eng.track_stats()
    print(f"tracks per stream: mean {st['T'].mean():.1f} max {st['T'].max()}; "
          f"{chk.n_dets} detections checked")
    assert st["overflow"].sum() == 0
    np.testing.assert_array_equal(st["T"], [len(t.tracks) for t in chk.trackers])
    assert chk.n_dets > 0
    eng.close()
