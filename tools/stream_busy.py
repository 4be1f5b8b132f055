"""Per-stream occupancy of bench.py's timed region from a rocprofv3 kernel
trace (the window between the two rv_trace_marker dispatches): for every
stream (Stream_Id, else Queue_Id) the kernels it ran, their summed time, the
union of its busy intervals and the idle gaps between consecutive kernels
(the launch / dependency-wait floor of that stream), per step; and which
kernel families sit next to the largest gaps.
usage: stream_busy.py kernel_trace.csv STEPS [A,B] > report.txt
(A,B: the marker tags of the window, default 1,2 = the timed region;
tools/trace_window.py lists bench.py's tags)"""
import csv
import gzip
import sys
from collections import defaultdict

from trace_window import CONV, family, marker_window


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = []
    for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        sid = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], sid,
                     int(r.get("Grid_Size_X") or 64) // 64))
    rows.sort()
    tags = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2").split(",")]
    a, b = marker_window([(r[0], r[1], r[2], r[4]) for r in rows], tags[0], tags[1])
    win = rows[a + 1:b]
    t0, t1 = rows[a][1], rows[b][0]
    wall = (t1 - t0) / steps / 1e3
    print(f"window: {len(win)} dispatches, {wall:.1f} us/step wall, chip busy (union of all) "
          f"{union([(s, e) for s, e, *_ in win]) / steps / 1e3:.1f} us/step")
    conv = [(s, e) for s, e, n, *_ in win if family(n) in CONV]
    print(f"conv family (conv_patch / conv1x1_direct / c2f_chain / stem): {len(conv) / steps:.2f} "
          f"launches/step, summed {sum(e - s for s, e in conv) / steps / 1e3:.1f} us/step, chip-union "
          f"busy {union(conv) / steps / 1e3:.1f} us/step")
    by = defaultdict(list)
    for r in win:
        by[r[3]].append(r)
    for sid, ks in sorted(by.items(), key=lambda t: -len(t[1])):
        ks.sort()
        dur = sum(e - s for s, e, *_ in ks)
        busy = union([(s, e) for s, e, *_ in ks])
        gaps = defaultdict(float)
        ngap = 0
        for (s0, e0, n0, *_), (s1, e1, n1, *_) in zip(ks, ks[1:]):
            g = s1 - e0
            if g > 0:
                gaps[(family(n0), family(n1))] += g
                ngap += 1
        fams = defaultdict(float)
        for s, e, n, *_ in ks:
            fams[family(n)] += e - s
        print(f"\nstream {sid}: {len(ks) / steps:.1f} kernels/step, summed {dur / steps / 1e3:.1f} "
              f"us/step, busy {busy / steps / 1e3:.1f} us/step ({busy / max(t1 - t0, 1):.1%} of wall), "
              f"gaps {sum(gaps.values()) / steps / 1e3:.1f} us/step")
        print("  kernels: " + ", ".join(f"{k} {v / steps / 1e3:.1f}" for k, v in
                                        sorted(fams.items(), key=lambda t: -t[1])[:8]))
        print("  largest gaps (after -> before, us/step): " + ", ".join(
            f"{a}->{b} {v / steps / 1e3:.1f}" for (a, b), v in
            sorted(gaps.items(), key=lambda t: -t[1])[:6]))


if __name__ == "__main__":
    main()
