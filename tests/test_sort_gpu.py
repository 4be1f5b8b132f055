"""SORT HIP kernel vs the reference's own trajectories (tests/golden) and the
oracle restatement.  Track ids / matches: exact.  distance_m: exact (f32).
speed_kmh: rel 1e-12 (f64 hypot).  KF state: rel 1e-9 (f64 matrices in a
different summation order than numpy's BLAS)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import sort_ref

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(GOLDEN, "reference_sort.npz"), allow_pickle=False)
CFG = {"max_staleness": 1.2, "min_hits": 3, "iou_threshold": 0.35, "speed_window": 0.8}


def _proj():
    from rvs_amd.geometry import HomographyProjector
    return HomographyProjector.from_matrix(G["proj/H"], G["proj/origin"],
                                           float(G["proj/max_distance"]))


def _run_streams(frames_per_stream, ts_per_stream, cfg, proj, cuda, dmax=128, tmax=1024):
    from rvs_amd.track.sort_hip import MultiStreamSort
    S = len(frames_per_stream)
    ms = MultiStreamSort(cfg, S, tmax=tmax, dmax=dmax, device=cuda)
    ms.set_projector(proj)
    nf = len(frames_per_stream[0])
    outs = [[] for _ in range(S)]
    for f in range(nf):
        dets = np.zeros((S, dmax, 6), np.float32)
        cnt = np.zeros(S, np.int32)
        ts = np.zeros(S, np.float64)
        for s in range(S):
            r = frames_per_stream[s][f]
            dets[s, :len(r)] = r
            cnt[s] = len(r)
            ts[s] = ts_per_stream[s][f]
        i, d, v = ms.update(torch.from_numpy(dets).to(cuda), torch.from_numpy(cnt).to(cuda),
                            torch.from_numpy(ts).to(cuda))
        i, d, v = i.cpu().numpy(), d.cpu().numpy(), v.cpu().numpy()
        for s in range(S):
            outs[s].append((i[s, :cnt[s]].copy(), d[s, :cnt[s]].copy(), v[s, :cnt[s]].copy()))
    return outs, ms


def _golden_traj(ti):
    rows, fr, ts = G[f"traj/{ti}/rows"], G[f"traj/{ti}/frame"], G[f"traj/{ti}/ts"]
    nf = int(G[f"traj/{ti}/nframes"])
    return [rows[fr == f] for f in range(nf)], list(ts), bool(G[f"traj/{ti}/proj"])


def _check(out, ti, nf=None):
    ids = np.concatenate([o[0] for o in out])
    dist = np.concatenate([o[1] for o in out])
    spd = np.concatenate([o[2] for o in out])
    n = len(ids)
    np.testing.assert_array_equal(ids, G[f"traj/{ti}/ids"][:n])
    np.testing.assert_array_equal(np.isnan(dist), np.isnan(G[f"traj/{ti}/dist"][:n]))
    np.testing.assert_array_equal(dist, G[f"traj/{ti}/dist"][:n])
    np.testing.assert_array_equal(np.isnan(spd), np.isnan(G[f"traj/{ti}/speed"][:n]))
    np.testing.assert_allclose(spd, G[f"traj/{ti}/speed"][:n], rtol=1e-12, equal_nan=True)


@pytest.mark.parametrize("ti", ["0", "1", "2"])
def test_reference_trajectory_single_stream(cuda, ti):
    frames, ts, use_proj = _golden_traj(ti)
    out, ms = _run_streams([frames], [ts], CFG, _proj() if use_proj else None, cuda)
    _check(out[0], ti)
    T, x, meta = ms.export()
    ref_ids = G[f"traj/{ti}/final_ids"]
    np.testing.assert_array_equal(meta[0, :T[0], 0], ref_ids)
    np.testing.assert_allclose(x[0, :T[0]], G[f"traj/{ti}/final_x"], rtol=1e-9, atol=1e-9)


def test_reference_trajectories_batched_streams(cuda):
    trajs = [_golden_traj(t) for t in ("0", "1", "2")]
    nf = min(len(t[0]) for t in trajs)
    # all three streams in one launch; projector on for all (traj 1 was
    # recorded without one, so compare ids only there)
    out, _ = _run_streams([t[0][:nf] for t in trajs], [t[1][:nf] for t in trajs], CFG, _proj(),
                          cuda)
    for s, ti in enumerate(("0", "1", "2")):
        ids = np.concatenate([o[0] for o in out[s]])
        np.testing.assert_array_equal(ids, G[f"traj/{ti}/ids"][:len(ids)])
        if ti != "1":
            _check(out[s], ti)


@pytest.mark.parametrize("thr,nobj", [(0.35, 60), (0.0, 70), (0.3, 5)])
def test_random_streams_vs_oracle(cuda, thr, nobj):
    cfg = dict(CFG, iou_threshold=thr)
    S, nf = 4, 80
    streams = [sort_ref.synthetic_detections(nf, seed=100 + s, n_obj=nobj, p_clutter=3.0)
               for s in range(S)]
    proj = _proj()
    out, _ = _run_streams([s[0] for s in streams], [s[1] for s in streams], cfg, proj, cuda)
    oproj = sort_ref.HomographyProjector(G["proj/H"], G["proj/origin"],
                                         float(G["proj/max_distance"]))
    for s in range(S):
        tr = sort_ref.SortTracker(cfg)
        for f in range(nf):
            dets = [sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in streams[s][0][f]]
            res = tr.update(dets, float(streams[s][1][f]), oproj)
            ids = [-1 if d.track_id is None else d.track_id for d in res]
            np.testing.assert_array_equal(out[s][f][0], ids, err_msg=f"stream {s} frame {f}")
            dd = [np.nan if d.distance_m is None else d.distance_m for d in res]
            np.testing.assert_array_equal(out[s][f][1], dd)


def test_tracker_api_semantics(cuda):
    from rvs_amd.detect import Detection
    from rvs_amd.track import build_tracker
    tr = build_tracker({"backend": "sort", **CFG})
    assert tr.update([], 0.0) == []
    d1 = [Detection(10, 10, 50, 60, 0.9, 2, "car"), Detection(200, 100, 260, 140, 0.8, 7, "truck")]
    out = tr.update(d1, 0.0)
    assert out[0] is d1[0] and [d.track_id for d in out] == [1, 2]
    d2 = [Detection(201, 101, 261, 141, 0.8, 7, "truck"), Detection(11, 10, 51, 61, 0.9, 2, "car")]
    assert [d.track_id for d in tr.update(d2, 1 / 30)] == [2, 1]
    d3 = [Detection(500, 500, 540, 560, 0.9, 2, "car")]
    assert [d.track_id for d in tr.update(d3, 5.0)] == [3]  # stale tracks pruned


def test_slot_reuse_and_capacity(cuda):
    """Track pool semantics: pruned tracks' slots are reused in the same frame
    (a stream creates far more tracks over time than tmax holds at once and
    still matches the reference), and exceeding tmax sets the stream's
    sticky overflow flag instead of failing silently."""
    cfg = dict(CFG, max_staleness=0.1)  # tracks die 3 frames after their last match
    S, nf, tmax = 2, 60, 24
    streams = [sort_ref.synthetic_detections(nf, seed=300 + s, n_obj=8, p_clutter=2.0)
               for s in range(S)]
    out, ms = _run_streams([s[0] for s in streams], [s[1] for s in streams], cfg, None, cuda,
                           tmax=tmax)
    st = ms.stats()
    assert st["overflow"].sum() == 0
    assert int(st["next_id"].min()) - 1 > tmax  # more tracks than slots over the run
    for s in range(S):
        tr = sort_ref.SortTracker(cfg)
        for f in range(nf):
            dets = [sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in streams[s][0][f]]
            res = tr.update(dets, float(streams[s][1][f]))
            ids = [-1 if d.track_id is None else d.track_id for d in res]
            np.testing.assert_array_equal(out[s][f][0], ids, err_msg=f"stream {s} frame {f}")
        assert int(st["T"][s]) == len(tr.tracks)
    # a pool too small for the live tracks: flagged, never silent
    out, ms = _run_streams([s[0] for s in streams], [s[1] for s in streams], CFG, None, cuda,
                           tmax=4)
    st = ms.stats()
    assert st["overflow"].all() and (st["T"] <= 4).all()
    from rvs_amd._lib import RVError
    with pytest.raises(RVError, match="capacity"):
        ms.check_capacity()
