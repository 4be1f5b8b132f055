"""Host cost of building the Detection lists of one 32-stream step
(rvs_amd.handback.to_detections) from a pinned host record versus from a
pageable copy of it: is the consumer bound by Python object creation or by
reads of pinned (hipHostMalloc) memory?  CPU-side only, but the record is
allocated with torch's pinned allocator (the GPU's host-memory path)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "road-vision-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rvs_amd.detect.weights import COCO80  # noqa: E402
from rvs_amd.handback import ROW, Record, to_detections  # noqa: E402

S, dmax, N = 32, 100, 50
rec = Record(S, dmax, "cuda")
n, rows = rec.arrays()
rng = np.random.default_rng(0)
for f in ("x1", "y1", "x2", "y2", "conf"):
    rows[f] = rng.uniform(0, 1000, (S, dmax))
rows["cls"] = rng.integers(0, 8, (S, dmax))
rows["track_id"] = rng.integers(-1, 400, (S, dmax))
rows["dist"] = np.where(rng.random((S, dmax)) < 0.5, np.nan, rng.uniform(0, 99, (S, dmax)))
rows["speed"] = np.nan
n[:] = 47


def timeit(fn):
    t = time.perf_counter()
    for _ in range(N):
        fn()
    return (time.perf_counter() - t) / N * 1e3


pinned = timeit(lambda: to_detections(*rec.arrays(), COCO80))
copy = timeit(lambda: rec.host.numpy().copy())
host = rec.host.numpy().copy()
hb = host[:4 * S].view(np.int32), host[(S * 4 + 15) & ~15:rec.nbytes].view(ROW).reshape(S, dmax)
pageable = timeit(lambda: to_detections(hb[0], hb[1], COCO80))
print(f"to_detections per step: pinned record {pinned:.3f} ms, pageable copy {pageable:.3f} ms "
      f"(copy itself {copy:.3f} ms), {int(n.sum())} detections", flush=True)
