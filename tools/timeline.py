"""Timeline statistics from a rocprofv3 kernel_trace.csv: over the last
`window` of the trace (default: everything after the last 10 % gap-free
region is ignored), the wall span, the sum of kernel durations, the time at
least one kernel was running (union) and the busy fraction -- i.e. how much
of a step is inter-kernel gap and whether kernels of different streams
overlap."""
import csv
import sys


def main():
    path = sys.argv[1]
    t0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # fraction of the trace to skip
    t1 = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    lo, hi = rows[0][0], max(r[1] for r in rows)
    a, b = lo + t0 * (hi - lo), lo + t1 * (hi - lo)
    sel = [r for r in rows if r[0] >= a and r[1] <= b]
    s = sum(r[1] - r[0] for r in sel)
    union, cur_s, cur_e = 0, None, None
    for st, en, _, _ in sel:
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    if cur_e is not None:
        union += cur_e - cur_s
    span = sel[-1][1] - sel[0][0] if sel else 0
    queues = sorted(set(r[3] for r in sel))
    print(f"kernels {len(sel)} span {span / 1e3:.1f} us sum {s / 1e3:.1f} us union {union / 1e3:.1f} us "
          f"busy {union / max(span, 1):.3f} overlap {s / max(union, 1):.3f} queues {queues}")


if __name__ == "__main__":
    main()
