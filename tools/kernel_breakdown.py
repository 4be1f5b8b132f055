"""Per-kernel-name time per step over the last N steps of a kernel trace
(steps delimited by clahe_lut_kernel launches)."""
import collections
import csv
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if "clahe_lut_kernel" in r[2]]
    sel = rows[idx[-n - 1]:idx[-1]]
    agg = collections.defaultdict(lambda: [0, 0])
    for st, en, name in sel:
        k = name.split("(")[0].replace("void ", "")[:60]
        agg[k][0] += 1
        agg[k][1] += en - st
    tot = sum(v[1] for v in agg.values())
    span = sel[-1][1] - sel[0][0]
    print(f"per step: kernel sum {tot / n / 1e3:.1f} us, span {span / n / 1e3:.1f} us")
    # idle time of the device (no kernel of any stream running) and the gaps
    # between consecutive YOLO kernels (dispatch latency on the critical path)
    union, cs, ce = 0, None, None
    gaps, ngap, prev_end = 0, 0, None
    for st, en, name in sel:
        if ce is None or st > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = st, en
        else:
            ce = max(ce, en)
        if "conv" in name or "stem" in name or "sppf" in name or "decode" in name:
            if prev_end is not None and 0 < st - prev_end < 20000:
                gaps += st - prev_end
                ngap += 1
            prev_end = en if prev_end is None else max(prev_end, en)
    union += ce - cs
    print(f"per step: device busy {union / n / 1e3:.1f} us (idle {(span - union) / n / 1e3:.1f} us); "
          f"gaps between YOLO kernels {gaps / n / 1e3:.1f} us over {ngap / n:.1f} launches")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{v[0] / n:5.1f} {v[1] / n / 1e3:8.1f} us {100 * v[1] / tot:5.1f}%  {k}")


if __name__ == "__main__":
    main()
