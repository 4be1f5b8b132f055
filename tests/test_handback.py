"""Host side of the result hand-back (rvs_amd.handback) on the CPU: the
column-wise to_detections builds exactly the Detection objects a row-by-row
construction does (src/detect/yolo_ultralytics.py:48-52 fields, then
sort_tracker.py:234-247's track_id / distance_m / speed_kmh; -1 / NaN ->
None), for ragged per-stream counts, empty streams, counts outside
[0, dmax] and class ids outside the name table."""
import math

import numpy as np

from rvs_amd.detect.types import Detection
from rvs_amd.detect.weights import COCO80
from rvs_amd.handback import ROW, to_detections


def _rowwise(n, rows, names):
    out = []
    for s in range(rows.shape[0]):
        lst = []
        for x1, y1, x2, y2, conf, k, tid, _, dist, spd in \
                rows[s, :max(0, min(int(n[s]), rows.shape[1]))].tolist():
            lst.append(Detection(x1, y1, x2, y2, conf, k,
                                 str(names[k]) if 0 <= k < len(names) else str(k),
                                 None if tid < 0 else tid,
                                 None if math.isnan(dist) else dist,
                                 None if math.isnan(spd) else spd))
        out.append(lst)
    return out


def test_to_detections_matches_rowwise_construction():
    rng = np.random.default_rng(7)
    S, dmax = 9, 17
    rows = np.zeros((S, dmax), ROW)
    for f in ("x1", "y1", "x2", "y2", "conf"):
        rows[f] = rng.uniform(-5, 2000, (S, dmax)).astype(np.float32)
    rows["cls"] = rng.integers(-2, 84, (S, dmax))
    rows["track_id"] = rng.integers(-1, 40, (S, dmax))
    rows["dist"] = np.where(rng.random((S, dmax)) < 0.3, np.nan, rng.uniform(0, 99, (S, dmax)))
    rows["speed"] = np.where(rng.random((S, dmax)) < 0.5, np.nan, rng.uniform(0, 150, (S, dmax)))
    n = np.array([0, 1, dmax, 5, -3, dmax + 4, 3, 16, 2], np.int32)
    got = to_detections(n, rows, COCO80)
    want = _rowwise(n, rows, COCO80)
    assert got == want
    assert [len(x) for x in got] == [0, 1, dmax, 5, 0, dmax, 3, 16, 2]
    for a, b in zip(sum(got, []), sum(want, [])):
        assert vars(a) == vars(b)
        assert all(type(getattr(a, f)) is type(getattr(b, f)) for f in vars(b))
    d = got[1][0]
    d.track_id = 5  # still an ordinary mutable Detection (SortTracker.update mutates it)
    assert d.track_id == 5 and isinstance(d, Detection)


def test_to_detections_empty():
    rows = np.zeros((3, 4), ROW)
    assert to_detections(np.zeros(3, np.int32), rows, COCO80) == [[], [], []]


def _record_bytes(n, rows):
    S, dmax = rows.shape
    hdr = (S * 4 + 15) & ~15
    buf = np.zeros(hdr + rows.nbytes, np.uint8)
    buf[:4 * S].view(np.int32)[:] = n
    buf[hdr:] = rows.reshape(-1).view(np.uint8)
    return buf


def test_c_builder_matches_python():
    """csrc/handback_py.c (Record.detections' builder) builds exactly the
    objects of to_detections from the raw record bytes (the 16-B-padded
    count header, then the 48-B rows)."""
    from rvs_amd import handback
    assert handback._rvhandback is not None, "the C builder is not built (make -C csrc)"
    rng = np.random.default_rng(11)
    for S, dmax in ((5, 9), (32, 100), (1, 1)):
        rows = np.zeros((S, dmax), ROW)
        for f in ("x1", "y1", "x2", "y2", "conf"):
            rows[f] = rng.uniform(-5, 2000, (S, dmax)).astype(np.float32)
        rows["cls"] = rng.integers(-2, 84, (S, dmax))
        rows["track_id"] = rng.integers(-1, 40, (S, dmax))
        rows["dist"] = np.where(rng.random((S, dmax)) < 0.3, np.nan, rng.uniform(0, 9, (S, dmax)))
        rows["speed"] = np.where(rng.random((S, dmax)) < 0.5, np.nan, rng.uniform(0, 9, (S, dmax)))
        n = rng.integers(-2, dmax + 3, S).astype(np.int32)
        got = handback._rvhandback.build(_record_bytes(n, rows), S, dmax, list(COCO80), Detection)
        want = to_detections(n, rows, COCO80)
        assert got == want
        for a, b in zip(sum(got, []), sum(want, [])):
            assert vars(a) == vars(b)
            assert all(type(getattr(a, f)) is type(getattr(b, f)) for f in vars(b))
    import pytest
    with pytest.raises(ValueError):
        handback._rvhandback.build(np.zeros(10, np.uint8), 2, 2, list(COCO80), Detection)


def test_c_builder_pool_shells():
    """Record.detections with a DetectionPool: the objects come from the
    pool's pre-made shells (consumed from its end; fresh ones once it runs
    out) and are exactly the objects of the plain build -- same fields,
    types and field order -- so a consumer may make them ahead of a
    hand-back (bench.py)."""
    from rvs_amd import handback
    assert handback._rvhandback is not None, "the C builder is not built (make -C csrc)"
    rng = np.random.default_rng(12)
    S, dmax = 6, 20
    rows = np.zeros((S, dmax), ROW)
    for f in ("x1", "y1", "x2", "y2", "conf"):
        rows[f] = rng.uniform(-5, 2000, (S, dmax)).astype(np.float32)
    rows["cls"] = rng.integers(-2, 84, (S, dmax))
    rows["track_id"] = rng.integers(-1, 40, (S, dmax))
    rows["dist"] = np.where(rng.random((S, dmax)) < 0.3, np.nan, rng.uniform(0, 9, (S, dmax)))
    rows["speed"] = np.where(rng.random((S, dmax)) < 0.5, np.nan, rng.uniform(0, 9, (S, dmax)))
    n = np.array([3, 0, 20, 7, -1, 25], np.int32)  # 50 detections
    rec = _record_bytes(n, rows)
    want = to_detections(n, rows, COCO80)
    for size in (0, 10, 50, 80):
        pool = handback.DetectionPool()
        pool.top_up(size)
        assert len(pool.items) == size
        assert all(isinstance(o, Detection) and list(vars(o)) == list(vars(want[0][0]))
                   and all(v is None for v in vars(o).values()) for o in pool.items)
        spare = list(pool.items[:max(0, size - 50)])
        got = handback._rvhandback.build(rec, S, dmax, list(COCO80), Detection, pool.items)
        assert got == want
        for a, b in zip(sum(got, []), sum(want, [])):
            assert vars(a) == vars(b) and list(vars(a)) == list(vars(b))
            assert all(type(getattr(a, f)) is type(getattr(b, f)) for f in vars(b))
        assert len(pool.items) == max(0, size - 50)
        assert all(x is y for x, y in zip(pool.items, spare))  # untouched shells stay
        ids = {id(o) for o in sum(got, [])}
        assert len(ids) == 50  # no object handed out twice


def _cpu_record(n, rows):
    """A Record over a plain CPU tensor (no pinned memory without a GPU)."""
    import torch
    from rvs_amd import handback
    S, dmax = rows.shape
    rec = object.__new__(handback.Record)
    rec.S, rec.dmax = S, dmax
    buf = _record_bytes(n, rows)
    rec.nbytes = buf.size
    rec.host = torch.from_numpy(buf)
    rec.seq = 0
    return rec


def _random_rows(rng, S, dmax):
    rows = np.zeros((S, dmax), ROW)
    for f in ("x1", "y1", "x2", "y2", "conf"):
        rows[f] = rng.uniform(-5, 2000, (S, dmax)).astype(np.float32)
    rows["cls"] = rng.integers(-2, 84, (S, dmax))
    rows["track_id"] = rng.integers(-1, 40, (S, dmax))
    rows["dist"] = np.where(rng.random((S, dmax)) < 0.3, np.nan, rng.uniform(0, 9, (S, dmax)))
    rows["speed"] = np.where(rng.random((S, dmax)) < 0.5, np.nan, rng.uniform(0, 9, (S, dmax)))
    return rows


def test_record_arrays_views_the_host_record():
    """Record.arrays() is a Record method (not DetectionPool's) and returns
    the count header and the 48-B rows of the host record."""
    from rvs_amd import handback
    assert hasattr(handback.Record, "arrays") and not hasattr(handback.DetectionPool, "arrays")
    rng = np.random.default_rng(21)
    rows = _random_rows(rng, 5, 7)
    n = np.array([1, 0, 7, 3, 9], np.int32)
    got_n, got_rows = _cpu_record(n, rows).arrays()
    assert got_n.tolist() == n.tolist()
    assert got_rows.tobytes() == rows.tobytes()


def test_record_detections_without_c_builder(monkeypatch):
    """With no C builder, Record.detections falls back to to_detections over
    Record.arrays() and gives the same objects as the C path."""
    from rvs_amd import handback
    rng = np.random.default_rng(22)
    rows = _random_rows(rng, 6, 11)
    n = np.array([0, 4, 11, 2, -1, 15], np.int32)
    rec = _cpu_record(n, rows)
    want = to_detections(n, rows, COCO80)
    c_built = rec.detections(COCO80) if handback._rvhandback is not None else want
    monkeypatch.setattr(handback, "_rvhandback", None)
    got = rec.detections(COCO80)
    assert got == want == c_built
    for a, b in zip(sum(got, []), sum(want, [])):
        assert vars(a) == vars(b)
