"""Ground-plane projection (mirrors src/geometry/projector.py:13-95).

Per-detection projection on the device happens inside the SORT kernel
(csrc/sort.hip: project / distance); this module keeps the reference's host
API (project_point / project_bbox / distance / distance_for_bbox) with the
same float64 / float32 arithmetic, and fits H at init.

cv2.findHomography(img_pts, world_pts) (method 0, projector.py:69) is
restated as the normalised DLT (Hartley normalisation, SVD null vector,
H /= H[2,2]); for exactly 4 correspondences this is the exact homography,
for N > 4 it is followed by Gauss-Newton refinement of the reprojection error
(OpenCV refines with Levenberg-Marquardt).  OpenCV is absent from this
environment, so H-fit parity against it is unpinned; per-detection
projection given H is pinned against the reference (tests/golden).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional, Sequence, Tuple

import numpy as np

Point2D = Tuple[float, float]


def find_homography(src: np.ndarray, dst: np.ndarray, refine_iters: int = 10) -> np.ndarray:
    src = np.asarray(src, np.float64).reshape(-1, 2)
    dst = np.asarray(dst, np.float64).reshape(-1, 2)

    def norm(p):
        c = p.mean(0)
        s = np.abs(p - c).mean(0)
        s[s == 0] = 1.0
        T = np.array([[1 / s[0], 0, -c[0] / s[0]], [0, 1 / s[1], -c[1] / s[1]], [0, 0, 1]])
        return T, (p - c) / s

    T1, a = norm(src)
    T2, b = norm(dst)
    n = a.shape[0]
    A = np.zeros((2 * n, 9))
    for i in range(n):
        x, y = a[i]
        u, v = b[i]
        A[2 * i] = [x, y, 1, 0, 0, 0, -u * x, -u * y, -u]
        A[2 * i + 1] = [0, 0, 0, x, y, 1, -v * x, -v * y, -v]
    _, _, vt = np.linalg.svd(A)
    Hn = vt[-1].reshape(3, 3)
    H = np.linalg.inv(T2) @ Hn @ T1
    if abs(H[2, 2]) < 1e-300:
        raise ValueError("degenerate homography")
    H = H / H[2, 2]
    if n > 4:
        h = H.ravel()[:8].copy()
        for _ in range(refine_iters):
            Hm = np.append(h, 1.0).reshape(3, 3)
            p = np.c_[src, np.ones(n)] @ Hm.T
            w = p[:, 2]
            r = np.concatenate([p[:, 0] / w - dst[:, 0], p[:, 1] / w - dst[:, 1]])
            J = np.zeros((2 * n, 8))
            x, y = src[:, 0], src[:, 1]
            J[:n, 0], J[:n, 1], J[:n, 2] = x / w, y / w, 1 / w
            J[n:, 3], J[n:, 4], J[n:, 5] = x / w, y / w, 1 / w
            J[:n, 6] = -p[:, 0] * x / w ** 2
            J[:n, 7] = -p[:, 0] * y / w ** 2
            J[n:, 6] = -p[:, 1] * x / w ** 2
            J[n:, 7] = -p[:, 1] * y / w ** 2
            step, *_ = np.linalg.lstsq(J, -r, rcond=None)
            h += step
            if np.abs(step).max() < 1e-12:
                break
        H = np.append(h, 1.0).reshape(3, 3)
    return H


class GroundProjector(ABC):
    def __init__(self, origin: Sequence[float] | None = None,
                 max_distance: float | None = None) -> None:
        if origin is None:
            origin = (0.0, 0.0)
        if len(origin) != 2:
            raise ValueError("origin must have length 2")
        self.origin = np.asarray(origin, dtype=np.float32)
        self.max_distance = float(max_distance) if max_distance is not None else None

    @abstractmethod
    def project_point(self, x: float, y: float) -> Optional[Point2D]:
        ...

    def project_bbox(self, bbox: Sequence[float]) -> Optional[Point2D]:
        x1, y1, x2, y2 = bbox
        return self.project_point(0.5 * (float(x1) + float(x2)), float(y2))

    def distance(self, point: Optional[Sequence[float]]) -> Optional[float]:
        if point is None:
            return None
        vec = np.asarray(point, dtype=np.float32) - self.origin
        dist = float(np.linalg.norm(vec))
        if not np.isfinite(dist):
            return None
        if self.max_distance is not None:
            dist = min(dist, self.max_distance)
        return dist

    def distance_for_bbox(self, bbox: Sequence[float]) -> Optional[float]:
        return self.distance(self.project_bbox(bbox))

    # device hand-off (the SORT kernel projects on the GPU)
    def device_params(self):
        """(H row-major f64[9], origin f32[2], max_distance or -1)."""
        raise NotImplementedError


class HomographyProjector(GroundProjector):
    def __init__(self, cfg: dict) -> None:
        super().__init__(origin=cfg.get("origin", (0.0, 0.0)), max_distance=cfg.get("max_distance"))
        img = np.asarray(cfg.get("image_points", []), dtype=np.float32)
        world = np.asarray(cfg.get("world_points", []), dtype=np.float32)
        if img.ndim != 2 or img.shape[0] < 4 or img.shape[1] != 2:
            raise ValueError("homography needs at least 4 image points (x, y)")
        if world.shape != img.shape:
            raise ValueError("image_points and world_points must have the same shape")
        self._H = find_homography(img, world).astype(np.float64)

    @classmethod
    def from_matrix(cls, H, origin=(0.0, 0.0), max_distance=None):
        self = cls.__new__(cls)
        GroundProjector.__init__(self, origin=origin, max_distance=max_distance)
        self._H = np.asarray(H, np.float64).reshape(3, 3)
        return self

    def project_point(self, x: float, y: float) -> Optional[Point2D]:
        pt = np.array([float(x), float(y), 1.0], dtype=np.float64)
        mapped = self._H @ pt
        w = float(mapped[2])
        if abs(w) < 1e-6:
            return None
        X = mapped[0] / w
        Y = mapped[1] / w
        if not (np.isfinite(X) and np.isfinite(Y)):
            return None
        return float(X), float(Y)

    def device_params(self):
        md = -1.0 if self.max_distance is None else float(self.max_distance)
        return self._H.ravel().astype(np.float64), self.origin.astype(np.float32), md


def build_projector(cfg: dict) -> GroundProjector:
    proj_cfg = cfg.get("projector") if isinstance(cfg, dict) else None
    if proj_cfg is None:
        proj_cfg = cfg
    proj_type = (proj_cfg.get("type") or "homography").lower()
    if proj_type == "homography":
        return HomographyProjector(proj_cfg)
    raise ValueError(f"unknown projector type: {proj_type}")
