"""Per-kernel statistics of bench.py's timed region from a rocprofv3 kernel
trace: keeps the dispatches between the two rv_trace_marker kernels bench.py
launches right before and right after its timed region (tags 1 and 2), so
warm-up, autotuning, capture and the CPU baseline are excluded.

usage: python tools/trace_window.py kernel_trace.csv STEPS OUT_PREFIX [A,B]
A,B (default 1,2) are the marker tags bracketing the window: the first
marker of tag A and the first marker of tag B after it.  rv_trace_marker
launches `tag` workgroups of 64, so a dispatch's tag is Grid_Size_X / 64.
bench.py's tags: 1,2 the timed region; 3,4 the in-pipeline conv profiling
pass; 5,6 the eager conv profiling pass (5 repetitions of every launch);
7,8 the device-only rerun of the timed region; 9,10 each warm run before it.
writes OUT_PREFIX_kernel_stats.csv (rocprofv3 --stats columns) and
OUT_PREFIX_summary.txt (per-step time of each kernel family, conv family
included, and the window's wall time)."""
import csv
import gzip
import sys
from collections import defaultdict

CONV = ("conv_patch_kernel", "conv1x1_direct_kernel", "c2f_chain_kernel", "stem_kernel")


def family(name: str) -> str:
    base = name.split("(")[0].replace("void ", "").strip()
    return base.split("<")[0].split("::")[-1]


def marker_window(rows, ta, tb):
    """Row indices of the first marker of tag ta and the first marker of tag
    tb after it (rows: (start, end, name, tag) sorted by start)."""
    marks = [(i, r[3]) for i, r in enumerate(rows) if "rv_trace_marker_kernel" in r[2]]
    a = next((i for i, t in marks if t == ta), None)
    b = next((i for i, t in marks if t == tb and a is not None and i > a), None)
    if a is None or b is None:
        sys.exit(f"no marker window {ta} -> {tb}: markers {[t for _, t in marks]}")
    return a, b


def main():
    path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    tags = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "1,2").split(",")]
    rows = []
    opener = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    for r in csv.DictReader(opener):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r.get("Grid_Size_X") or 64) // 64))
    rows.sort()
    a, b = marker_window(rows, tags[0], tags[1])
    win = rows[a + 1:b]
    t0, t1 = rows[a][1], rows[b][0]
    agg = defaultdict(list)
    for s, e, n, _ in win:
        agg[n].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    with open(out + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                    "MaxNs"])
        for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, len(v), sum(v), sum(v) / len(v), round(100 * sum(v) / tot, 2),
                        min(v), max(v)])
    fam = defaultdict(lambda: [0, 0])
    for n, v in agg.items():
        f_ = family(n)
        fam[f_][0] += len(v)
        fam[f_][1] += sum(v)
    conv_ns = sum(sum(v) for n, v in agg.items() if any(c in n for c in CONV))
    conv_calls = sum(len(v) for n, v in agg.items() if any(c in n for c in CONV))
    with open(out + "_summary.txt", "w") as f:
        f.write(f"timed-region window: {len(win)} dispatches, wall {(t1 - t0) / 1e6:.3f} ms "
                f"over {steps} steps = {(t1 - t0) / 1e3 / steps:.1f} us/step\n")
        f.write(f"conv family: {conv_calls} launches ({conv_calls / steps:.1f}/step), "
                f"{conv_ns / 1e3 / steps:.1f} us/step summed kernel time, avg "
                f"{conv_ns / max(conv_calls, 1) / 1e3:.2f} us/launch\n")
        f.write(f"{'family':40s} {'calls/step':>10s} {'us/step':>9s} {'avg_us':>8s}\n")
        for f_, (c, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
            f.write(f"{f_[:40]:40s} {c / steps:10.2f} {ns / 1e3 / steps:9.1f} {ns / c / 1e3:8.2f}\n")
    print(open(out + "_summary.txt").read())


if __name__ == "__main__":
    main()
