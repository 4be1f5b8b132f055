"""First repetition vs the warm ones in bench.py's eager conv pass (trace
window tags 5-6: every conv launch of a unit issued 5 times back to back
between its HIP events): from a rocprofv3 kernel trace, the conv-family
dispatches are cut into consecutive runs of REPS (5), each checked to be
one launch repeated (same kernel, grid), and the first dispatch of each run (inputs as the forward
leaves them) is summed apart from repetitions 2-5 (inputs warm in L2 /
MALL from the repetition before).
usage: python tools/eager_reps.py kernel_trace.csv[.gz] STEPS [GFLOP_PER_STEP [REPS]]"""
import csv
import gzip
import sys

from trace_window import CONV, family, marker_window


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    gflop = float(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = []
    for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r.get("Grid_Size_X") or 64) // 64, r.get("Grid_Size_Y", "")))
    rows.sort()
    a, b = marker_window([r[:4] for r in rows], 5, 6)
    win = [r for r in rows[a + 1:b] if family(r[2]) in CONV]
    R = int(sys.argv[4]) if len(sys.argv) > 4 else 5  # bench.py's eager repetitions
    if len(win) % R:
        sys.exit(f"{len(win)} conv dispatches in the window: not runs of {R}")
    first = warm = 0.0
    nfirst = nwarm = 0
    for g in range(0, len(win), R):
        run = win[g:g + R]
        if len({(r[2], r[3], r[4]) for r in run}) != 1:
            sys.exit(f"dispatches {g}..{g + R - 1} are not one launch repeated")
        first += run[0][1] - run[0][0]
        nfirst += 1
        for s, e, *_ in run[1:]:
            warm += e - s
            nwarm += 1
    reps = R
    f_us = first / 1e3 / steps
    w_us = warm / 1e3 / steps / max(reps - 1, 1)
    print(f"{nfirst} runs of {reps:.2f} repetitions: first repetition {f_us:.1f} us per step, "
          f"a warm repetition {w_us:.1f} us per step ({f_us / w_us:.3f}x)")
    if gflop:
        for lab, us in (("first", f_us), ("warm", w_us)):
            tf = gflop / (us * 1e-6) / 1e3
            print(f"  {lab}: {tf:.1f} TFLOP/s = {tf / 2500:.4f} of the 2.5 PF bf16 peak")


if __name__ == "__main__":
    main()
