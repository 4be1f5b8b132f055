"""Generate golden vectors from the REFERENCE's own code (run in the build
container, where /root/reference is mounted read-only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's SORT and geometry modules import cv2 and filterpy at module
level (src/geometry/projector.py:7, src/track/sort_tracker.py:9-12); both are
absent here (ordinary ImportError, not a permission denial).
They are satisfied with stand-ins that the exercised code never calls into
(cv2: only findHomography at HomographyProjector.__init__, bypassed by
setting _H directly) or that restate the third-party algorithm (filterpy's
KalmanFilter -> oracle.sort_ref.KalmanFilter).  Everything else -- _iou,
_iou_matrix, _associate, _bbox_to_z, _x_to_bbox, _Track, SortTracker.update,
GroundProjector / HomographyProjector.project_point -- is the reference code
running unmodified.  Output: tests/golden/reference_sort.npz (data only).
"""
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

from oracle import sort_ref  # noqa: E402

REF = "/root/reference"


def import_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    fp = types.ModuleType("filterpy")
    fpk = types.ModuleType("filterpy.kalman")
    fpk.KalmanFilter = sort_ref.KalmanFilter
    fp.kalman = fpk
    sys.modules["filterpy"] = fp
    sys.modules["filterpy.kalman"] = fpk
    sys.path.insert(0, REF)
    from src.track import sort_tracker as st
    from src.geometry import projector as pj
    from src.detect.types import Detection
    return st, pj, Detection


def rand_boxes(rng, n, degenerate=False):
    x1 = rng.uniform(0, 500, n)
    y1 = rng.uniform(0, 300, n)
    w = rng.uniform(1, 120, n)
    h = rng.uniform(1, 120, n)
    b = np.stack([x1, y1, x1 + w, y1 + h], 1).astype(np.float32)
    if degenerate and n > 3:
        b[0, 2] = b[0, 0]          # zero width
        b[1, 3] = b[1, 1] - 5      # negative height
        b[2] = b[3]                # duplicate (ties)
    return b


def main():
    st, pj, Detection = import_reference()
    rng = np.random.default_rng(1234)
    out = {}

    # 1. _iou_matrix, incl. empty and degenerate boxes
    cases = [(0, 5), (5, 0), (1, 1), (7, 9), (30, 30), (64, 100)]
    for ci, (T, D) in enumerate(cases):
        tb = rand_boxes(rng, T, degenerate=True)
        db = np.concatenate([tb[: min(T, D) // 2] + rng.normal(0, 3, (min(T, D) // 2, 4)).astype(
            np.float32), rand_boxes(rng, D - min(T, D) // 2, degenerate=True)]).astype(np.float32)
        out[f"iou/{ci}/trk"] = tb
        out[f"iou/{ci}/det"] = db
        out[f"iou/{ci}/out"] = st._iou_matrix(tb, db)

    # 2. _associate (greedy argmax) with ties and several thresholds
    class FakeTrack:
        def __init__(self, b):
            self.b = b

        def get_state(self):
            return self.b

    acase = 0
    for T, D in [(5, 5), (12, 9), (40, 35), (3, 8)]:
        for thr in (0.35, 0.3, 0.0, 0.9):
            tb = rand_boxes(rng, T)
            idx = rng.permutation(T)[: min(T, D)]
            db = np.concatenate([tb[idx] + rng.normal(0, 4, (len(idx), 4)).astype(np.float32),
                                 rand_boxes(rng, D - len(idx))]).astype(np.float32)
            if T >= 3 and D >= 3:
                db[1] = db[0]  # exact tie between two detections
            tr = st.SortTracker({"iou_threshold": thr})
            tr._tracks = [FakeTrack(b) for b in tb]
            dets = [Detection(*map(float, b), 0.5, 2, "car") for b in db]
            m, ut, ud = tr._associate(dets)
            out[f"assoc/{acase}/trk"] = tb
            out[f"assoc/{acase}/det"] = db
            out[f"assoc/{acase}/thr"] = np.array(thr)
            out[f"assoc/{acase}/matches"] = np.array(m, np.int64).reshape(-1, 2)
            out[f"assoc/{acase}/ut"] = np.array(sorted(ut), np.int64)
            out[f"assoc/{acase}/ud"] = np.array(sorted(ud), np.int64)
            acase += 1

    # 3. _bbox_to_z / _x_to_bbox
    bb = np.concatenate([rand_boxes(rng, 50), np.array([[5, 5, 5, 5], [10, 10, 9, 8]], np.float32)])
    out["z/in"] = bb
    out["z/out"] = np.stack([st._bbox_to_z(tuple(map(float, b))).reshape(-1) for b in bb])
    xs = np.concatenate([rng.normal(0, 1, (40, 7)) * [300, 200, 5000, 0.5, 3, 3, 50] +
                         [600, 400, 8000, 1.2, 0, 0, 0], [[1, 1, -5, 2, 0, 0, 0]]])
    out["x/in"] = xs
    out["x/out"] = np.stack([st._x_to_bbox(x.reshape(7, 1)) for x in xs])

    # 4. projector
    H = np.array([[0.02, 0.001, -19.0], [0.0005, -0.05, 60.0], [1e-5, 0.0012, 1.0]], np.float64)
    proj = pj.HomographyProjector.__new__(pj.HomographyProjector)
    pj.GroundProjector.__init__(proj, origin=(0.5, -2.0), max_distance=80.0)
    proj._H = H
    pb = np.concatenate([rand_boxes(rng, 200) * 3, np.array([[0, -1e9, 1, -833.33], [0, 0, 0, 0]],
                                                            np.float32)])
    pts, dist = [], []
    for b in pb:
        p = proj.project_bbox(tuple(map(float, b)))
        pts.append([np.nan, np.nan] if p is None else list(p))
        d = proj.distance_for_bbox(tuple(map(float, b)))
        dist.append(np.nan if d is None else d)
    out["proj/H"] = H
    out["proj/origin"] = np.array([0.5, -2.0], np.float32)
    out["proj/max_distance"] = np.array(80.0)
    out["proj/boxes"] = pb
    out["proj/points"] = np.array(pts, np.float64)
    out["proj/dist"] = np.array(dist, np.float64)

    # 5. SortTracker.update trajectories (reference control flow end to end)
    cfg = {"max_staleness": 1.2, "min_hits": 3, "iou_threshold": 0.35, "speed_window": 0.8}
    for ti, (use_proj, seed, nf, nobj) in enumerate([(True, 7, 90, 12), (False, 8, 60, 25),
                                                     (True, 9, 45, 40)]):
        frames, ts = sort_ref.synthetic_detections(nf, seed=seed, n_obj=nobj)
        # a gap longer than max_staleness, and an empty frame
        ts = [t + (2.0 if i >= nf // 2 else 0.0) for i, t in enumerate(ts)]
        frames[nf // 3] = frames[nf // 3][:0]
        tr = st.SortTracker(cfg)
        ids, dd, sp, fidx, rows = [], [], [], [], []
        for f, (rows_f, t) in enumerate(zip(frames, ts)):
            dets = [Detection(*map(float, r[:5]), int(r[5]), "c") for r in rows_f]
            res = tr.update(dets, float(t), proj if use_proj else None)
            for d, r in zip(res, rows_f):
                ids.append(-1 if d.track_id is None else d.track_id)
                dd.append(np.nan if d.distance_m is None else d.distance_m)
                sp.append(np.nan if d.speed_kmh is None else d.speed_kmh)
                fidx.append(f)
                rows.append(r)
        out[f"traj/{ti}/rows"] = np.array(rows, np.float32).reshape(-1, 6)
        out[f"traj/{ti}/frame"] = np.array(fidx, np.int64)
        out[f"traj/{ti}/ts"] = np.array(ts, np.float64)
        out[f"traj/{ti}/nframes"] = np.array(nf)
        out[f"traj/{ti}/proj"] = np.array(use_proj)
        out[f"traj/{ti}/ids"] = np.array(ids, np.int64)
        out[f"traj/{ti}/dist"] = np.array(dd, np.float64)
        out[f"traj/{ti}/speed"] = np.array(sp, np.float64)
        out[f"traj/{ti}/final_x"] = np.stack([t.kf.x.reshape(-1) for t in tr._tracks]) \
            if tr._tracks else np.zeros((0, 7))
        out[f"traj/{ti}/final_ids"] = np.array([t.id for t in tr._tracks], np.int64)
    out["traj/cfg"] = np.array([cfg["max_staleness"], cfg["min_hits"], cfg["iou_threshold"],
                                cfg["speed_window"]])
    path = os.path.join(HERE, "reference_sort.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
