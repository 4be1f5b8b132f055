"""Standalone tracker / geometry entries (csrc/track_ops.hip) against the
vectors the reference's own code produced (tests/golden/make_golden.py:
_iou_matrix, _associate, GroundProjector).  Bit-exact: IoU values, match
lists in acceptance order, unmatched lists.  Projection: the reference's
`H @ [x, y, 1]` goes through numpy's matvec, whose summation order differs
from the kernel's scalar f64 expression, and the terms can cancel, so points
are asserted to rtol 1e-12 / atol 1e-12 (measured: 7e-15 abs at worst) and
the f32 distances to 1 f32 ulp ("<= 1 ulp f64 (numpy
matvec order)").
All golden cases run as ONE batch of streams (padded to Tmax x Dmax)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import sort_ref

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(GOLDEN, "reference_sort.npz"), allow_pickle=False)


def _keys(prefix):
    return sorted({k.split("/")[1] for k in G.files if k.startswith(prefix + "/")
                   and k.split("/")[1].isdigit()}, key=int)


def _pack(cases, cuda):
    S = len(cases)
    Tm = max(1, max(len(t) for t, _ in cases))
    Dm = max(1, max(len(d) for _, d in cases))
    trk = np.zeros((S, Tm, 4), np.float32)
    det = np.zeros((S, Dm, 4), np.float32)
    for s, (t, d) in enumerate(cases):
        trk[s, :len(t)] = t
        det[s, :len(d)] = d
    T = torch.tensor([len(t) for t, _ in cases], dtype=torch.int32, device=cuda)
    D = torch.tensor([len(d) for _, d in cases], dtype=torch.int32, device=cuda)
    return torch.from_numpy(trk).to(cuda), T, torch.from_numpy(det).to(cuda), D


def test_iou_matrix_batched_matches_reference(cuda):
    from rvs_amd.track.sort_hip import iou_matrix_batched
    ids = _keys("iou")
    cases = [(G[f"iou/{i}/trk"].reshape(-1, 4), G[f"iou/{i}/det"].reshape(-1, 4)) for i in ids]
    trk, T, det, D = _pack(cases, cuda)
    out = iou_matrix_batched(trk, T, det, D).cpu().numpy()
    for s, i in enumerate(ids):
        ref = G[f"iou/{i}/out"]
        nt, nd = len(cases[s][0]), len(cases[s][1])
        np.testing.assert_array_equal(out[s, :nt, :nd], ref.reshape(nt, nd))
        assert not out[s, nt:].any() and not out[s, :, nd:].any()


def test_greedy_assign_batched_matches_reference(cuda):
    from rvs_amd.track.sort_hip import associate_batched, iou_matrix_batched
    ids = _keys("assoc")
    by_thr = {}
    for i in ids:  # one launch per threshold value (the threshold is per call)
        by_thr.setdefault(float(G[f"assoc/{i}/thr"]), []).append(i)
    for thr, grp in by_thr.items():
        cases = [(G[f"assoc/{i}/trk"].reshape(-1, 4), G[f"assoc/{i}/det"].reshape(-1, 4))
                 for i in grp]
        trk, T, det, D = _pack(cases, cuda)
        M = iou_matrix_batched(trk, T, det, D)
        mt, md, n, tm, dm = [x.cpu().numpy() for x in associate_batched(M, T, D, thr)]
        for s, i in enumerate(grp):
            ref = [tuple(r) for r in G[f"assoc/{i}/matches"].tolist()]
            got = list(zip(mt[s, :n[s]].tolist(), md[s, :n[s]].tolist()))
            assert got == ref, (i, thr)
            nt, nd = len(cases[s][0]), len(cases[s][1])
            assert [t for t in range(nt) if tm[s, t] < 0] == G[f"assoc/{i}/ut"].tolist()
            assert [d for d in range(nd) if dm[s, d] < 0] == G[f"assoc/{i}/ud"].tolist()


def test_homography_project_matches_reference(cuda):
    from rvs_amd.track.sort_hip import project_boxes
    H = torch.from_numpy(np.ascontiguousarray(G["proj/H"], np.float64)).to(cuda)
    boxes = torch.from_numpy(np.ascontiguousarray(G["proj/boxes"], np.float32)).to(cuda)
    origin = torch.from_numpy(np.ascontiguousarray(G["proj/origin"], np.float32)).to(cuda)
    xy, dist = project_boxes(H, boxes, origin, float(G["proj/max_distance"]))
    xy, dist = xy.cpu().numpy(), dist.cpu().numpy()
    ref_xy, ref_d = G["proj/points"], G["proj/dist"]
    np.testing.assert_array_equal(np.isnan(xy), np.isnan(ref_xy))  # None cases
    np.testing.assert_allclose(xy, ref_xy, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(np.isnan(dist), np.isnan(ref_d))
    ok = ~np.isnan(ref_d)
    ulp = np.spacing(ref_d[ok].astype(np.float32)).astype(np.float64)
    assert (np.abs(dist[ok] - ref_d[ok]) <= ulp).all()
    print("exact distances:", float((dist[ok] == ref_d[ok]).mean()))


def test_update_many_matches_single_stream_trackers(cuda):
    from rvs_amd.detect.types import Detection
    from rvs_amd.config import load_config
    from rvs_amd.track.sort_hip import MultiStreamSort
    cfg = load_config()["tracking"]
    S, F = 3, 5
    core = MultiStreamSort(cfg, S)
    refs = [sort_ref.SortTracker(cfg) for _ in range(S)]
    rng = np.random.default_rng(2)
    base = rng.uniform(0, 300, (S, 4, 2))
    for f in range(F):
        frames = [[Detection(x + 3 * f, y, x + 3 * f + 40, y + 30, 0.8, 2, "car")
                   for x, y in base[s][: 2 + (f + s) % 3]] for s in range(S)]
        out = core.update_many(frames, [f / 30.0] * S)
        for s in range(S):
            dets = [sort_ref.Det(d.x1, d.y1, d.x2, d.y2, d.conf, d.cls_id) for d in frames[s]]
            refs[s].update(dets, f / 30.0)
            assert [d.track_id for d in out[s]] == [d.track_id for d in dets]
