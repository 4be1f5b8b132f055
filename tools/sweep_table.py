"""Best forced tile per conv position from tools/conv_sweep.sh traces."""
import glob
import os
import sqlite3
import sys

PERIOD = 66


def per_pos(db, reps=3):
    global PERIOD
    c = sqlite3.connect(db)
    rows = list(c.execute("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d join "
                          "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    # period = launches per forward: distance between the last two conv0 launches
    idx = [i for i, r in enumerate(rows) if "conv0_kernel" in r[0]]
    PERIOD = idx[-1] - idx[-2]
    tail = rows[idx[-reps]:idx[-reps] + PERIOD * reps]
    return [(tail[i][0], sum(tail[r * PERIOD + i][1] for r in range(reps)) / reps / 1e3)
            for i in range(PERIOD)]


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--dump":  # on the box: trace dir -> small text table
        dbs = glob.glob(os.path.join(sys.argv[2], "**", "*.db"), recursive=True)
        for name, t in per_pos(dbs[0]):
            print(f"{t:.3f} {name}")
        return
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep"
    res = {}
    for f in sorted(glob.glob(os.path.join(root, "*_p*.txt"))):
        rows = [ln.split(" ", 1) for ln in open(f).read().splitlines() if ln.strip()]
        res[os.path.basename(f)[:-4]] = [(n, float(t)) for t, n in rows]
    base = res.get("auto_p1")
    tot_auto = sum(t for n, t in base)
    best_tot = 0.0
    for i in range(PERIOD):
        name = base[i][0]
        if "conv_patch" not in name:
            best_tot += base[i][1]
            continue
        cands = sorted((v[i][1], k) for k, v in res.items() if "conv_patch" in v[i][0])
        best_tot += cands[0][0]
        print(f"{i:3d} auto {base[i][1]:7.2f}  best {cands[0][0]:7.2f} {cands[0][1]:10s} "
              f"2nd {cands[1][0]:7.2f} {cands[1][1]}")
    print(f"forward kernel sum: auto {tot_auto:.1f} us, per-layer best {best_tot:.1f} us")


if __name__ == "__main__":
    main()
