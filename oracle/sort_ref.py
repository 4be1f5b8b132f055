"""Python/numpy restatement of the reference SORT tracker and ground projector
-- TEST INFRASTRUCTURE ONLY (checker + bench cpu_baseline leg).

Follows src/track/sort_tracker.py:22-281 and src/geometry/projector.py:13-84
line by line, with filterpy's KalmanFilter (filterpy ~1.4.5, absent from
this container, unpinned in requirements.txt:6) restated from its published
predict/update equations:
    predict: x = F x ; P = alpha^2 * F P F^T + Q            (alpha = 1)
    update:  y = z - H x ; PHT = P H^T ; S = H PHT + R ; SI = inv(S)
             K = PHT SI ; x = x + K y ; I_KH = I - K H
             P = I_KH P I_KH^T + K R K^T                     (Joseph form)
with the same numpy.dot call structure so results are bit-identical to
filterpy on the same numpy/BLAS.  The restatement is pinned against vectors
the reference code itself produced (tests/golden/make_golden.py), where the
reference's own SortTracker runs with this KalmanFilter in place of
filterpy.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np


class KalmanFilter:
    """filterpy.kalman.KalmanFilter subset used by sort_tracker.py."""

    def __init__(self, dim_x: int, dim_z: int):
        self.dim_x, self.dim_z = dim_x, dim_z
        self.x = np.zeros((dim_x, 1))
        self.P = np.eye(dim_x)
        self.Q = np.eye(dim_x)
        self.F = np.eye(dim_x)
        self.H = np.zeros((dim_z, dim_x))
        self.R = np.eye(dim_z)
        self._alpha_sq = 1.0
        self._I = np.eye(dim_x)

    def predict(self):
        self.x = np.dot(self.F, self.x)
        self.P = self._alpha_sq * np.dot(np.dot(self.F, self.P), self.F.T) + self.Q

    def update(self, z):
        z = np.asarray(z).reshape(self.dim_z, 1) if np.ndim(z) != 2 else z
        H, R = self.H, self.R
        y = z - np.dot(H, self.x)
        PHT = np.dot(self.P, H.T)
        S = np.dot(H, PHT) + R
        SI = np.linalg.inv(S)
        K = np.dot(PHT, SI)
        self.x = self.x + np.dot(K, y)
        I_KH = self._I - np.dot(K, H)
        self.P = np.dot(np.dot(I_KH, self.P), I_KH.T) + np.dot(np.dot(K, R), K.T)


def bbox_to_z(bbox):
    x1, y1, x2, y2 = bbox
    w = max(1e-3, float(x2) - float(x1))
    h = max(1e-3, float(y2) - float(y1))
    cx = float(x1) + 0.5 * w
    cy = float(y1) + 0.5 * h
    return np.array([[cx], [cy], [w * h], [w / h]], dtype=np.float32)


def x_to_bbox(state):
    cx, cy, s, r = state[:4].reshape(-1)
    w = math.sqrt(max(1e-6, s * r))
    h = s / max(1e-6, w)
    return np.array([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], dtype=np.float32)


def iou(a, b):
    ax1, ay1, ax2, ay2 = a
    bx1, by1, bx2, by2 = b
    iw = max(0.0, min(ax2, bx2) - max(ax1, bx1))
    ih = max(0.0, min(ay2, by2) - max(ay1, by1))
    inter = iw * ih
    area_a = max(0.0, ax2 - ax1) * max(0.0, ay2 - ay1)
    area_b = max(0.0, bx2 - bx1) * max(0.0, by2 - by1)
    denom = area_a + area_b - inter
    if denom <= 0.0:
        return 0.0
    return float(inter / denom)


def iou_matrix(tb: np.ndarray, db: np.ndarray) -> np.ndarray:
    out = np.zeros((tb.shape[0], db.shape[0]), dtype=np.float32)
    if tb.size == 0 or db.size == 0:
        return out
    for i, t in enumerate(tb):
        for j, d in enumerate(db):
            out[i, j] = iou(t, d)
    return out


def greedy(m: np.ndarray, thr: float):
    """sort_tracker.py:190-210 on a (T, D) f32 matrix (destroyed)."""
    matches = []
    ut = set(range(m.shape[0]))
    ud = set(range(m.shape[1]))
    if m.size == 0:
        return matches, list(ut), list(ud)
    while True:
        idx = int(np.argmax(m))
        if float(m.flat[idx]) < thr:
            break
        t, d = np.unravel_index(idx, m.shape)
        if t in ut and d in ud:
            matches.append((int(t), int(d)))
            ut.remove(int(t))
            ud.remove(int(d))
        m[t, :] = -1.0
        m[:, d] = -1.0
    return matches, list(ut), list(ud)


class HomographyProjector:
    """projector.py:13-84 with H given (findHomography is init-only)."""

    def __init__(self, H, origin=(0.0, 0.0), max_distance=None):
        self._H = np.asarray(H, dtype=np.float64).reshape(3, 3)
        self.origin = np.asarray(origin, dtype=np.float32)
        self.max_distance = float(max_distance) if max_distance is not None else None

    def project_point(self, x, y):
        mapped = self._H @ np.array([float(x), float(y), 1.0], dtype=np.float64)
        w = float(mapped[2])
        if abs(w) < 1e-6:
            return None
        X, Y = mapped[0] / w, mapped[1] / w
        if not (np.isfinite(X) and np.isfinite(Y)):
            return None
        return float(X), float(Y)

    def project_bbox(self, bbox):
        x1, y1, x2, y2 = bbox
        return self.project_point(0.5 * (float(x1) + float(x2)), float(y2))

    def distance(self, point):
        if point is None:
            return None
        d = float(np.linalg.norm(np.asarray(point, dtype=np.float32) - self.origin))
        if not np.isfinite(d):
            return None
        if self.max_distance is not None:
            d = min(d, self.max_distance)
        return d

    def distance_for_bbox(self, bbox):
        return self.distance(self.project_bbox(bbox))


@dataclass
class Det:
    x1: float
    y1: float
    x2: float
    y2: float
    conf: float
    cls_id: int
    cls_name: str = ""
    track_id: Optional[int] = None
    distance_m: Optional[float] = None
    speed_kmh: Optional[float] = None


class _Track:
    def __init__(self, tid, bbox, ts, min_hits, speed_window):
        self.id = tid
        kf = KalmanFilter(dim_x=7, dim_z=4)
        kf.F = np.eye(7, dtype=float)
        kf.H = np.zeros((4, 7), dtype=float)
        kf.H[:4, :4] = np.eye(4, dtype=float)
        kf.R[2:, 2:] *= 10.0
        kf.P[4:, 4:] *= 1000.0
        kf.P *= 10.0
        self.kf = kf
        self._motion(1.0)
        self.kf.x[:4, 0] = bbox_to_z(bbox).reshape(-1)
        self.last_predict_ts = float(ts)
        self.last_update_ts = float(ts)
        self.min_hits = max(1, int(min_hits))
        self.speed_window = max(0.05, float(speed_window))
        self.hits = 1
        self.hit_streak = 1
        self.hist: List[Tuple[float, float, float]] = []
        self.current_distance = None
        self.current_speed = None
        self.class_id = None
        self.confidence = None

    def _motion(self, dt):
        dt = float(max(1e-3, dt))
        F = np.eye(7, dtype=float)
        F[0, 4] = F[1, 5] = F[2, 6] = dt
        self.kf.F = F
        q = np.zeros((7, 7), dtype=float)
        q[0, 0] = q[1, 1] = q[2, 2] = 0.04 * dt * dt
        q[4, 4] = q[5, 5] = q[6, 6] = 1.0 * dt
        self.kf.Q = q

    def predict(self, ts):
        self._motion(float(ts) - self.last_predict_ts)
        self.kf.predict()
        self.last_predict_ts = float(ts)
        return x_to_bbox(self.kf.x)

    def update(self, bbox, ts, det):
        self._motion(float(ts) - self.last_predict_ts)
        self.kf.update(bbox_to_z(bbox))
        self.last_predict_ts = float(ts)
        self.last_update_ts = float(ts)
        self.hits += 1
        self.hit_streak += 1
        self.class_id = det.cls_id
        self.confidence = det.conf

    def update_metrics(self, proj, bbox, ts):
        g = proj.project_bbox(bbox)
        if g is None:
            self.current_distance = None
            self.current_speed = None
            return
        self.current_distance = proj.distance(g)
        self.hist.append((float(ts), float(g[0]), float(g[1])))
        while self.hist and (float(ts) - self.hist[0][0]) > self.speed_window:
            self.hist.pop(0)
        if len(self.hist) > 32:
            self.hist = self.hist[-32:]
        if len(self.hist) >= 2:
            t0, x0, y0 = self.hist[0]
            t1, x1, y1 = self.hist[-1]
            self.current_speed = math.hypot(x1 - x0, y1 - y0) / max(1e-3, t1 - t0)
        else:
            self.current_speed = None


class SortTracker:
    def __init__(self, cfg):
        self.max_staleness = float(cfg.get("max_staleness", 1.0))
        self.min_hits = int(cfg.get("min_hits", 3))
        self.iou_threshold = float(cfg.get("iou_threshold", 0.3))
        self.speed_window = float(cfg.get("speed_window", 0.75))
        self.tracks: List[_Track] = []
        self.next_id = 1

    def update(self, dets: Sequence[Det], ts: float, proj=None):
        dets = list(dets)
        for d in dets:
            d.track_id = d.distance_m = d.speed_kmh = None
        if not dets and not self.tracks:
            return dets
        for t in self.tracks:
            t.predict(ts)
        if not self.tracks or not dets:
            matches, ut, ud = [], list(range(len(self.tracks))), list(range(len(dets)))
        else:
            tb = np.array([x_to_bbox(t.kf.x) for t in self.tracks], dtype=np.float32)
            db = np.array([[d.x1, d.y1, d.x2, d.y2] for d in dets], dtype=np.float32)
            matches, ut, ud = greedy(iou_matrix(tb, db), self.iou_threshold)
        for ti, di in matches:
            t, d = self.tracks[ti], dets[di]
            bb = (d.x1, d.y1, d.x2, d.y2)
            t.update(bb, ts, d)
            if proj is not None:
                t.update_metrics(proj, bb, ts)
            d.track_id = t.id
            if t.current_distance is not None:
                d.distance_m = t.current_distance
            elif proj is not None:
                d.distance_m = proj.distance_for_bbox(bb)
            if t.current_speed is not None:
                d.speed_kmh = t.current_speed * 3.6
        for ti in ut:
            self.tracks[ti].hit_streak = 0
        for di in ud:
            d = dets[di]
            bb = (d.x1, d.y1, d.x2, d.y2)
            t = _Track(self.next_id, bb, ts, self.min_hits, self.speed_window)
            t.class_id, t.confidence = d.cls_id, d.conf
            if proj is not None:
                t.update_metrics(proj, bb, ts)
                if t.current_distance is not None:
                    d.distance_m = t.current_distance
                if t.current_speed is not None:
                    d.speed_kmh = t.current_speed * 3.6
            d.track_id = t.id
            self.tracks.append(t)
            self.next_id += 1
        self.tracks = [t for t in self.tracks if float(ts) - t.last_update_ts <= self.max_staleness]
        return dets


def synthetic_detections(n_frames: int, seed: int = 0, n_obj: int = 20, W=1920, H=1080,
                         fps=30.0, p_miss=0.1, p_clutter=2.0):
    """Drifting boxes with misses and clutter: per frame a list of
    (x1,y1,x2,y2,conf,cls) float32 rows, plus timestamps."""
    rng = np.random.default_rng(seed)
    cx = rng.uniform(100, W - 100, n_obj)
    cy = rng.uniform(200, H - 100, n_obj)
    w = rng.uniform(40, 200, n_obj)
    h = w * rng.uniform(0.6, 1.2, n_obj)
    vx = rng.uniform(-6, 6, n_obj)
    vy = rng.uniform(-2, 4, n_obj)
    cls = rng.choice([0, 2, 3, 5, 7], n_obj)
    frames, ts = [], []
    for f in range(n_frames):
        rows = []
        for i in range(n_obj):
            if rng.uniform() < p_miss:
                continue
            jx, jy = rng.normal(0, 1.5, 2)
            rows.append([cx[i] - w[i] / 2 + jx, cy[i] - h[i] / 2 + jy, cx[i] + w[i] / 2 + jx,
                         cy[i] + h[i] / 2 + jy, rng.uniform(0.3, 0.95), cls[i]])
        for _ in range(rng.poisson(p_clutter)):
            x0, y0 = rng.uniform(0, W - 50), rng.uniform(0, H - 50)
            s = rng.uniform(20, 80)
            rows.append([x0, y0, x0 + s, y0 + s, rng.uniform(0.26, 0.5), rng.choice([0, 2])])
        rng.shuffle(rows)
        frames.append(np.array(rows, np.float32).reshape(-1, 6))
        ts.append(f / fps + rng.normal(0, 0.002))
        cx += vx
        cy += vy
        out = (cx < -100) | (cx > W + 100) | (cy > H + 100)
        cx[out] = rng.uniform(100, W - 100, out.sum())
        cy[out] = rng.uniform(200, 400, out.sum())
    return frames, ts
