"""Capture front end (rv_capture_*, rvs_amd.io_video) on the CPU: the native
reader threads, the YUV4MPEG2 parser and its I420 -> NV12 interleave, raw
formats, in-order slots, end of stream, looping and read timestamps
(src/io_video/capture.py:10-24).  No GPU calls: the slots are pageable host
memory when no HIP device is present."""
import ctypes
import time

import numpy as np
import pytest

from conftest import road_frame


def _frames(n, H=48, W=64):
    return [road_frame(H, W, seed=300 + i) for i in range(n)]


def _i420_planes(path):
    """Independent parse of a y4m file: list of (Y, U, V) planes."""
    data = open(path, "rb").read()
    hdr, rest = data.split(b"\n", 1)
    toks = hdr.split()
    W = int([t for t in toks if t.startswith(b"W")][0][1:])
    H = int([t for t in toks if t.startswith(b"H")][0][1:])
    out = []
    while rest:
        line, rest = rest.split(b"\n", 1)
        assert line.startswith(b"FRAME")
        ny, nc = W * H, W * H // 4
        buf = np.frombuffer(rest[:ny + 2 * nc], np.uint8)
        rest = rest[ny + 2 * nc:]
        out.append((buf[:ny].reshape(H, W), buf[ny:ny + nc].reshape(H // 2, W // 2),
                    buf[ny + nc:].reshape(H // 2, W // 2)))
    return out, W, H


def _reader(path, fmt, W=0, H=0, nbuf=3, loop=False):
    from rvs_amd.io_video.capture import _Reader
    return _Reader(str(path), fmt, W, H, nbuf, loop)


def test_y4m_reader_hands_out_nv12_in_order(tmp_path):
    from rvs_amd.io_video import write_y4m
    p = tmp_path / "cam.y4m"
    write_y4m(str(p), _frames(7))
    planes, W, H = _i420_planes(p)
    r = _reader(p, 0, nbuf=3)
    assert (r.W, r.H, r.frame_bytes, r.pinned) == (W, H, W * H * 3 // 2, 0)
    t_prev = 0.0
    for i, (y, u, v) in enumerate(planes):
        ptr, ts, idx, slot = r.next()
        got = np.ctypeslib.as_array((ctypes.c_uint8 * r.frame_bytes).from_address(ptr)).copy()
        assert idx == i and ts >= t_prev and abs(ts - time.time()) < 60
        t_prev = ts
        np.testing.assert_array_equal(got[:W * H].reshape(H, W), y)
        uv = got[W * H:].reshape(H // 2, W // 2, 2)
        np.testing.assert_array_equal(uv[..., 0], u)
        np.testing.assert_array_equal(uv[..., 1], v)
        r.release(slot)
    assert r.next() is None and r.next() is None  # end of stream stays ended
    r.close()


def test_raw_formats_loop_and_held_slots(tmp_path):
    H, W = 10, 12
    fr = [np.full((H, W, 3), i, np.uint8) for i in range(5)]
    p = tmp_path / "cam.bgr"
    p.write_bytes(b"".join(f.tobytes() for f in fr))
    r = _reader(p, 2, W, H, nbuf=2, loop=True)
    seen, held = [], []
    for k in range(12):  # loops over the 5 frames; hold two slots at a time
        ptr, ts, idx, slot = r.next()
        v = np.ctypeslib.as_array((ctypes.c_uint8 * r.frame_bytes).from_address(ptr))
        seen.append((idx, int(v[0])))
        held.append(slot)
        if len(held) == 2:
            r.release(held.pop(0))
    assert [i for i, _ in seen] == list(range(12))
    assert [v for _, v in seen] == [k % 5 for k in range(12)]
    r.close()
    # NV12 raw: a truncated trailing frame ends the stream
    q = tmp_path / "cam.nv12"
    q.write_bytes(bytes(range(256)) * 3 + b"\x01" * 5)  # 768 B = 4 frames of 8x16 + 5 B
    r = _reader(q, 1, 16, 8, nbuf=4)
    n = 0
    while (got := r.next()) is not None:
        r.release(got[3])
        n += 1
    assert n == 4
    r.close()


def test_capture_errors(tmp_path):
    from rvs_amd import _lib
    from rvs_amd.io_video import VideoSource
    bad = tmp_path / "x.y4m"
    bad.write_bytes(b"YUV4MPEG2 W64 H48 C444\nFRAME\n")
    with pytest.raises(_lib.RVError, match="4:2:0"):
        _reader(bad, 0)
    with pytest.raises(_lib.RVError, match="cannot open"):
        _reader(tmp_path / "missing.y4m", 0)
    with pytest.raises(_lib.RVError, match="nbuf"):
        _reader(bad, 0, nbuf=1)
    with pytest.raises(NotImplementedError):
        VideoSource(0)
    with pytest.raises(ValueError, match="unsupported"):
        VideoSource(str(tmp_path / "clip.mp4"))
    lib = _lib.load()
    assert lib.rv_capture_release(None, 0) == -1000 and lib.rv_capture_close(None) == 0
