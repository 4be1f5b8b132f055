"""Per-position kernel durations of a repeated launch sequence from a
rocprofv3 rocpd database: the last `reps` repetitions of a period-`n` launch
sequence are averaged position by position (e.g. the ~70 launches of one
YOLOv8 forward)."""
import sqlite3
import sys


def main():
    db, period, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, d.start, d.end, d.grid_size_x, d.grid_size_y from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    rows = list(c.execute(q))
    tail = rows[len(rows) - period * reps:]
    tot = 0.0
    out = []
    for i in range(period):
        ds = [tail[r * period + i][2] - tail[r * period + i][1] for r in range(reps)]
        name, _, _, gx, gy = tail[i]
        avg = sum(ds) / reps / 1e3
        tot += avg
        out.append((i, avg, gx, gy, name))
    span = (tail[-1][2] - tail[0][1]) / reps / 1e3
    print(f"sum of kernel averages {tot:.1f} us per sequence, wall span {span:.1f} us")
    for i, avg, gx, gy, name in out:
        print(f"{i:3d} {avg:8.2f} us grid {gx:8d}x{gy:<4d} {name[:90]}")


if __name__ == "__main__":
    main()
