"""Integration: the batched engine (preprocess -> detect -> track -> hand-back)
checked stage by stage against the oracle fed with the GPU's own upstream
outputs: proc frames bit-exact; NMS exact on the GPU's raw prediction (the
same kernel sequence as the candidate path); SORT ids / distances exact and
speeds to 1e-9 relative on the GPU's detections; no stream overflows tmax.

test_bench_configuration_parity runs exactly what bench.py times: 32
streams of 1080p, per-layer autotuned conv kernels, the 4-stage software
pipeline issued by the native launch list (rvs_amd.schedule.PipelinedRun),
results handed back to pinned host records inside the step (reference call
order: main_preview.py:94-109)."""
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


@pytest.mark.parametrize("mode,sync,pair,units,after_stem", [
    ("native", "flow", 1, None, "1"), ("native", "stage", 1, None, "1"),
    ("native", "flow", 2, None, "1"), ("native", "stage", 2, None, "1"),
    ("eager", "flow", 2, None, "1"), ("eager", "stage", 1, None, "1"),
    ("native", "flow", 4, [1, 2, 4, 1], "1"), ("eager", "flow", 2, [1, 1, 2, 2, 1, 1], "1"),
    ("native", "flow", 2, None, "0"), ("eager", "flow", 4, [4, 2, 2], "0")])
def test_pipelined_run_matches_sequential_steps(cuda, monkeypatch, mode, sync, pair, units,
                                                after_stem):
    """bench.py's timed mode (rvs_amd.schedule.PipelinedRun): units of `pair`
    steps software-pipelined over four HIP streams -- preprocess of unit u+1,
    the two forward halves of units u and u-1 on two lanes, NMS + SORT +
    hand-back of unit u-2 -- issued by the native launch list or eagerly,
    lock-stepped or chained by per-dependency events; `units`: unequal unit
    sizes (bench.py --units ramp: short units at both ends); `after_stem`:
    the next unit's preprocess waits for forward part 3 of the current one
    (the default; "0" = one part 1, the r03 order).  EVERY step's
    handed-back detections / track ids and proc frames, and the final SORT
    state, must equal those of plain sequential step() calls; a second run()
    of the same schedule continues the tracks like K more step() calls."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    monkeypatch.setenv("RV_PREP_AFTER_STEM", after_stem)
    cfg = _cfg()
    S, H, W = 4, 1080, 1920
    K = 8  # a multiple of pair
    F = 1 + 2 * K
    frames = road_frames(S, F, H, W, device=cuda)
    ts = torch.tensor([[f / 30.0] * S for f in range(F)], dtype=torch.float64, device=cuda)
    seq = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    seq_res, seq_proc = [], []
    for f in range(F):
        out_seq = seq.step(frames[f], ts[f])
        seq_res.append(seq.results(out_seq))
        seq_proc.append(out_seq["proc"].cpu().numpy())
    pip = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=2, pair=pair)
    pip.step(frames[0], ts[0])
    key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id, d.distance_m,  # noqa
                       d.speed_kmh) for d in s] for s in r]
    for r in range(2):  # two runs over two windows of K steps
        f0 = 1 + r * K
        run = PipelinedRun(pip, [frames[f0 + k] for k in range(K)],
                           [ts[f0 + k] for k in range(K)], mode=mode, sync=sync, units=units)
        if mode == "native":
            assert run.sched.num_nodes() > 0
        run.run()
        torch.cuda.synchronize()
        assert len(run.outs) == K
        for k, o in enumerate(run.outs):
            assert key(seq_res[f0 + k]) == key(pip.results(o)), f"run {r} step {k}"
            np.testing.assert_array_equal(o["proc"].cpu().numpy(), seq_proc[f0 + k])
        run.close()
    Ts, xs, ms = seq.tracker.export()
    To, xo, mo = pip.tracker.export()
    np.testing.assert_array_equal(Ts, To)
    for s in range(S):
        np.testing.assert_array_equal(xs[s, :Ts[s]], xo[s, :To[s]])
        np.testing.assert_array_equal(ms[s, :Ts[s]], mo[s, :To[s]])
    seq.close()
    pip.close()


def test_native_schedule_replays(cuda):
    """The same recorded launch list run twice over the same inputs: the
    second run continues SORT from the first (ids keep counting) and its
    preprocess / detections equal a fresh eager pipeline's second run."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W, K = 2, 720, 1280, 4
    frames = road_frames(S, K, H, W, device=cuda)
    ts = [torch.full((S,), k / 30.0, dtype=torch.float64, device=cuda) for k in range(K)]
    outs = {}
    for mode in ("native", "eager"):
        eng = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=2, pair=2)
        run = PipelinedRun(eng, [frames[k] for k in range(K)], ts, mode=mode)
        got = []
        for _ in range(2):
            run.run()
            torch.cuda.synchronize()
            got.append([eng.results(o) for o in run.outs])
        key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id)  # noqa
                          for d in s] for s in r]
        outs[mode] = [[key(r) for r in g] for g in got]
        run.close()
        eng.close()
    assert outs["native"] == outs["eager"]
    ids0 = {d[6] for st in outs["native"][0] for s in st for d in s if d[6] is not None}
    ids1 = {d[6] for st in outs["native"][1] for s in st for d in s if d[6] is not None}
    assert ids0 and ids1


def test_native_schedule_keeps_temporaries_and_checks_runs(cuda):
    """A recorded node holds raw device pointers: the schedule must keep the
    temporaries made while recording alive (here the .contiguous() copies of
    stream-interleaved frame views), so runs after the memory was churned
    still read the right frames.  rv_sched_event_sync refuses an event
    before the first run (no stale or unwritten record is ever handed out)."""
    from rvs_amd._lib import RVError
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W, K = 2, 720, 1280, 2
    frames = road_frames(S, K, H, W, device=cuda)
    ts = [torch.full((S,), k / 30.0, dtype=torch.float64, device=cuda) for k in range(K)]
    # (H, S, W, 3) storage viewed as (S, H, W, 3): not the ABI's pitch layout
    views = []
    for k in range(K):
        inter = torch.empty((H, S, W, 3), dtype=torch.uint8, device=cuda)
        inter.copy_(frames[k].permute(1, 0, 2, 3))
        views.append(inter.permute(1, 0, 2, 3))
    assert not views[0].is_contiguous()
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=2, pair=2)
    run = PipelinedRun(eng, views, ts, mode="native")
    with pytest.raises(RVError):
        run.wait_step(0)  # no run yet
    with pytest.raises(RVError):
        run.step_ready(0)  # the non-blocking form, same rule
    torch.cuda.synchronize()
    churn = [torch.full((S, H, W, 3), 7, dtype=torch.uint8, device=cuda) for _ in range(4)]
    run.run()
    while not run.step_ready(K - 1):
        pass
    run.wait_step(K - 1)
    torch.cuda.synchronize()
    for k, o in enumerate(run.outs):
        src = frames[k].cpu().numpy()
        pr = o["proc"].cpu().numpy()
        for s in range(S):
            np.testing.assert_array_equal(pr[s], cpu.median(cpu.clahe_ycrcb(src[s]), 3))
    del churn
    run.close()
    eng.close()


@pytest.mark.parametrize("pair", [1, 4])
def test_bench_configuration_parity(cuda, pair):
    """Exactly bench.py's timed configuration (S = 32 streams of 1080p,
    autotuned conv kernels on persistent grids, PipelinedRun native launch
    list with per-dependency events on two forward lanes, hand-back into
    per-step host records), checked against the oracle on every step:
    proc bit-exact on a sample of streams, NMS exact on the GPU's raw
    prediction for all 32 streams, SORT ids / distances exact for all 32
    streams, and no stream ever exceeds tmax."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    S, H, W, WARM, K = 32, 1080, 1920, 2, 8
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=2, pair=pair)
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
    run = PipelinedRun(eng, [frames[WARM + k] for k in range(K)],
                       [ts[WARM + k] for k in range(K)], mode="native", sync="flow")
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
    run.close()
    eng.close()


def test_forward_part4_continues_part3(cuda):
    """rv_yolo_forward_part part 4 (model.3 .. model.15) must continue the
    handle's last part 3 (stem, model.2) with the same batch and workspace:
    refused before any part 3 and for another batch."""
    from rvs_amd._lib import RVError
    from rvs_amd.engine import RoadVisionEngine
    eng = RoadVisionEngine(_cfg(), 2, (720, 1280), device=cuda, lanes=2, pair=2)
    det = eng.detector
    lb = det.lb[0][:4]
    with pytest.raises(RVError):
        det.forward_raw(lb, lane=0, part=4)
    det.forward_raw(lb, lane=0, part=3)
    with pytest.raises(RVError):
        det.forward_raw(det.lb[0][:2], lane=0, part=4)
    det.forward_raw(lb, lane=0, part=4)
    det.forward_raw(None, lane=0, part=2, batch=4)
    # a bare part 3 invalidates the earlier part 1 / 4: part 2 needs the part 4
    # that continues it, never the stale model.3 .. model.15 activations
    det.forward_raw(lb, lane=0, part=3)
    with pytest.raises(RVError):
        det.forward_raw(None, lane=0, part=2, batch=4)
    det.forward_raw(lb, lane=0, part=4)
    det.forward_raw(None, lane=0, part=2, batch=4)
    torch.cuda.synchronize()
    eng.close()


def _untracked_oracle(eng, cfg, proc, proj):
    """Oracle detections of one step with the tracker off: the oracle NMS of
    the GPU's own raw prediction, then main_preview.py:104-109 (distance_for_bbox
    per detection when a projector exists; ids and speeds stay None)."""
    raw = torch.empty((eng.S, 84, eng.detector.A), dtype=torch.float32, device=eng.device)
    eng.detector.set_raw_fused(True)
    eng.detector.forward_raw(eng.detector.letterbox(proc), raw, candidates=False)
    eng.detector.set_raw_fused(False)
    ref = yolo_ref.postprocess(raw.cpu().numpy(), (eng.detector.in_h, eng.detector.in_w),
                               (eng.H, eng.W), classes_keep=cfg["detect"]["classes_keep"])
    out = []
    for s in range(eng.S):
        lst = []
        for r in ref[s]:
            x1, y1, x2, y2, conf = map(float, r[:5])
            dist = proj.distance_for_bbox((x1, y1, x2, y2)) if proj is not None else None
            lst.append((x1, y1, x2, y2, conf, int(r[5]), None, dist, None))
        out.append(lst)
    return out


@pytest.mark.parametrize("geometry", [True, False])
def test_tracking_disabled_matches_oracle(cuda, geometry):
    """tracking.enabled false (main_preview.py:64-70,101-109): no SORT runs;
    every Detection keeps track_id / speed_kmh None and, with geometry on,
    gets distance_m = projector.distance_for_bbox(bbox) -- compared field by
    field with the oracle (boxes, conf, class exact; distances bit-exact)."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    cfg["tracking"]["enabled"] = False
    cfg["geometry"]["enabled"] = geometry
    S, H, W, F = 3, 1080, 1920, 3
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    assert eng.tracker is None
    proj = sort_ref.HomographyProjector(eng.projector._H, (0.0, 0.0), 1000.0) if geometry else None
    frames = road_frames(S, F, H, W, device=cuda)
    n = 0
    for f in range(F):
        out = eng.step(frames[f], torch.full((S,), f / 30.0, dtype=torch.float64, device=cuda))
        res = eng.results(out)
        want = _untracked_oracle(eng, cfg, out["proc"], proj)
        got = [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id, d.distance_m, d.speed_kmh)
                for d in s] for s in res]
        # boxes / conf compared as the f32 values the reference's floats come from
        for gs, ws in zip(got, want):
            assert len(gs) == len(ws)
            for g, w in zip(gs, ws):
                assert np.float32(g[:5]).tobytes() == np.float32(w[:5]).tobytes()
                assert g[5:] == w[5:]
                assert g[6] is None and g[8] is None
                assert (g[7] is None) == (not geometry)
        n += sum(len(s) for s in res)
    assert n > 0
    eng.close()


def test_tracking_disabled_pipelined_equals_steps(cuda):
    """The pipelined native schedule with the tracker off (rv_untracked_metrics
    recorded as a node) hands back exactly what sequential step() calls do."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    cfg["tracking"]["enabled"] = False
    S, H, W, K = 2, 1080, 1920, 4
    frames = road_frames(S, K, H, W, device=cuda)
    ts = [torch.full((S,), k / 30.0, dtype=torch.float64, device=cuda) for k in range(K)]
    seq = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    key = lambda r: [[(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id, d.track_id, d.distance_m,  # noqa
                       d.speed_kmh) for d in s] for s in r]
    want = [key(seq.results(seq.step(frames[k], ts[k]))) for k in range(K)]
    pip = RoadVisionEngine(cfg, S, (H, W), device=cuda, lanes=2, pair=2)
    run = PipelinedRun(pip, [frames[k] for k in range(K)], ts, mode="native")
    run.run()
    torch.cuda.synchronize()
    for k, o in enumerate(run.outs):
        assert key(pip.results(o)) == want[k]
    assert any(d[7] is not None for r in want for s in r for d in s)
    run.close()
    seq.close()
    pip.close()


def test_detection_disabled_returns_empty_lists(cuda):
    """detect.enabled false (main_preview.py:60-62,97-99): no detector is
    built, the preprocess still produces proc (bit-exact), and every
    stream's list is empty."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.schedule import PipelinedRun
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    cfg["detect"]["enabled"] = False
    S, H, W = 2, 720, 1280
    eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    assert eng.detector is None and eng.tracker is None
    frames = road_frames(S, 2, H, W, device=cuda)
    out = eng.step(frames[0], torch.zeros(S, dtype=torch.float64, device=cuda))
    assert eng.results(out) == [[], []]
    src = frames[0].cpu().numpy()
    pr = out["proc"].cpu().numpy()
    for s in range(S):
        np.testing.assert_array_equal(pr[s], cpu.median(cpu.clahe_ycrcb(src[s]), 3))
    with pytest.raises(ValueError):
        PipelinedRun(eng, [frames[0]], [torch.zeros(S, dtype=torch.float64, device=cuda)])
    eng.close()


def test_projector_build_failure_runs_without_geometry(cuda):
    """geometry.enabled with only 2 image points: the projector fails to
    build, the engine warns and runs on without it (main_preview.py:72-78),
    so SORT still assigns ids and every distance / speed stays None."""
    from rvs_amd.engine import RoadVisionEngine
    from rvs_amd.synth import road_frames
    cfg = _cfg()
    cfg["geometry"]["projector"]["image_points"] = IMG[:2]
    cfg["geometry"]["projector"]["world_points"] = WLD[:2]
    S, H, W = 2, 1080, 1920
    with pytest.warns(UserWarning, match="projector"):
        eng = RoadVisionEngine(cfg, S, (H, W), device=cuda)
    assert eng.projector is None and eng.tracker is not None
    frames = road_frames(S, 2, H, W, device=cuda)
    n = 0
    for f in range(2):
        res = eng.results(eng.step(frames[f], torch.full((S,), f / 30.0, dtype=torch.float64,
                                                         device=cuda)))
        for s in res:
            for d in s:
                assert d.track_id is not None
                assert d.distance_m is None and d.speed_kmh is None
                n += 1
    assert n > 0
    eng.close()
