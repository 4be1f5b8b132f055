"""Pin the SORT / geometry oracle against vectors produced by the reference's
own code (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import cpu, sort_ref

G = np.load(os.path.join(GOLDEN, "reference_sort.npz"), allow_pickle=False)


def keys(prefix):
    return sorted({k.split("/")[1] for k in G.files if k.startswith(prefix + "/")
                   and k.split("/")[1].isdigit()}, key=int)


@pytest.mark.parametrize("ci", keys("iou"))
def test_iou_matrix_c_and_python_match_reference(ci):
    tb, db, ref = G[f"iou/{ci}/trk"], G[f"iou/{ci}/det"], G[f"iou/{ci}/out"]
    np.testing.assert_array_equal(cpu.iou_matrix(tb, db), ref)
    np.testing.assert_array_equal(sort_ref.iou_matrix(tb, db), ref)


@pytest.mark.parametrize("ai", keys("assoc"))
def test_greedy_association_matches_reference(ai):
    tb, db = G[f"assoc/{ai}/trk"], G[f"assoc/{ai}/det"]
    thr = float(G[f"assoc/{ai}/thr"])
    ref = [tuple(r) for r in G[f"assoc/{ai}/matches"].tolist()]
    assert cpu.greedy(cpu.iou_matrix(tb, db), thr) == ref
    m, ut, ud = sort_ref.greedy(sort_ref.iou_matrix(tb, db), thr)
    assert m == ref
    assert sorted(ut) == G[f"assoc/{ai}/ut"].tolist()
    assert sorted(ud) == G[f"assoc/{ai}/ud"].tolist()


def test_bbox_state_conversions_match_reference():
    z = np.stack([sort_ref.bbox_to_z(tuple(map(float, b))).reshape(-1) for b in G["z/in"]])
    np.testing.assert_array_equal(z, G["z/out"])
    x = np.stack([sort_ref.x_to_bbox(s.reshape(7, 1)) for s in G["x/in"]])
    np.testing.assert_array_equal(x, G["x/out"])


def test_projector_matches_reference():
    p = sort_ref.HomographyProjector(G["proj/H"], G["proj/origin"], float(G["proj/max_distance"]))
    for b, pt, d in zip(G["proj/boxes"], G["proj/points"], G["proj/dist"]):
        got = p.project_bbox(tuple(map(float, b)))
        if np.isnan(pt[0]):
            assert got is None
        else:
            assert got == (pt[0], pt[1])
        gd = p.distance_for_bbox(tuple(map(float, b)))
        assert (gd is None and np.isnan(d)) or gd == d


def test_distance_is_plain_f32_sum_of_squares():
    """The GPU kernel computes sqrtf(vx*vx + vy*vy) in f32 without FMA; the
    reference's np.linalg.norm on a float32 2-vector gives the same bits."""
    o = G["proj/origin"]
    md = float(G["proj/max_distance"])
    for pt, d in zip(G["proj/points"], G["proj/dist"]):
        if np.isnan(pt[0]):
            continue
        v = np.asarray(pt, np.float32) - o
        s = np.float32(v[0] * v[0]) + np.float32(v[1] * v[1])
        mine = min(float(np.sqrt(np.float32(s))), md)
        assert mine == d


@pytest.mark.parametrize("ti", keys("traj"))
def test_sort_trajectory_matches_reference(ti):
    if ti == "cfg":
        return
    c = G["traj/cfg"]
    cfg = {"max_staleness": c[0], "min_hits": int(c[1]), "iou_threshold": c[2],
           "speed_window": c[3]}
    proj = sort_ref.HomographyProjector(G["proj/H"], G["proj/origin"],
                                        float(G["proj/max_distance"])) \
        if bool(G[f"traj/{ti}/proj"]) else None
    rows, fr, ts = G[f"traj/{ti}/rows"], G[f"traj/{ti}/frame"], G[f"traj/{ti}/ts"]
    tr = sort_ref.SortTracker(cfg)
    ids, dd, sp = [], [], []
    for f in range(int(G[f"traj/{ti}/nframes"])):
        dets = [sort_ref.Det(*map(float, r[:5]), int(r[5])) for r in rows[fr == f]]
        for d in tr.update(dets, float(ts[f]), proj):
            ids.append(-1 if d.track_id is None else d.track_id)
            dd.append(np.nan if d.distance_m is None else d.distance_m)
            sp.append(np.nan if d.speed_kmh is None else d.speed_kmh)
    np.testing.assert_array_equal(ids, G[f"traj/{ti}/ids"])
    np.testing.assert_array_equal(np.array(dd), G[f"traj/{ti}/dist"])
    np.testing.assert_array_equal(np.array(sp), G[f"traj/{ti}/speed"])
    np.testing.assert_array_equal([t.id for t in tr.tracks], G[f"traj/{ti}/final_ids"])
