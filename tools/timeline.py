"""Timeline of a bench.py trace window (rocprofv3 kernel trace): the window
between two rv_trace_marker dispatches cut into bins, and per bin the chip's
busy fraction (union of all kernel intervals) and the kernel-family time in
it (summed over streams, so > 1 when families overlap).  Shows where the
pipeline fills and drains: bins at the start / end of the window whose
families are one stage only.
usage: timeline.py kernel_trace.csv[.gz] [A,B] [BIN_US] > report.txt"""
import csv
import gzip
import sys
from collections import defaultdict

from trace_window import family, marker_window


def main():
    path = sys.argv[1]
    tags = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2").split(",")]
    bin_ns = int(float(sys.argv[3]) * 1e3) if len(sys.argv) > 3 else 250_000
    rows = []
    for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r.get("Grid_Size_X") or 64) // 64))
    rows.sort()
    a, b = marker_window(rows, tags[0], tags[1])
    t0, t1 = rows[a][1], rows[b][0]
    win = [r for r in rows[a + 1:b]]
    nb = (t1 - t0 + bin_ns - 1) // bin_ns
    fam = [defaultdict(float) for _ in range(nb)]
    busy = [[] for _ in range(nb)]
    for s, e, name, _ in win:
        s, e = max(s, t0), min(e, t1)
        f = family(name)
        k = (s - t0) // bin_ns
        while k < nb and t0 + k * bin_ns < e:
            lo, hi = max(s, t0 + k * bin_ns), min(e, t0 + (k + 1) * bin_ns)
            if hi > lo:
                fam[k][f] += (hi - lo) / bin_ns
                busy[k].append((lo, hi))
            k += 1
    print(f"window tags {tags[0]},{tags[1]}: {(t1 - t0) / 1e6:.3f} ms, {len(win)} dispatches, "
          f"bins of {bin_ns / 1e3:.0f} us")
    print("bin   t_ms   busy  families (summed stream-time / bin)")
    tot_idle = 0.0
    for k in range(nb):
        iv = sorted(busy[k])
        u, cs, ce = 0, None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    u += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        u += (ce - cs) if ce is not None else 0
        width = min(bin_ns, t1 - (t0 + k * bin_ns))
        frac = u / width if width > 0 else 0.0
        tot_idle += (1 - frac) * width
        top = sorted(fam[k].items(), key=lambda x: -x[1])[:5]
        print(f"{k:3d} {k * bin_ns / 1e6:6.2f}  {frac:5.2f}  " +
              "  ".join(f"{n} {v:.2f}" for n, v in top))
    print(f"idle (no kernel running): {tot_idle / 1e6:.3f} ms of {(t1 - t0) / 1e6:.3f}")


if __name__ == "__main__":
    main()
