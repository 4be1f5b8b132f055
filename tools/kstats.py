"""Per-kernel duration summary from a rocprofv3 rocpd SQLite database or a
kernel_trace.csv (used to read the profiles under gpurun_out/ / profiles/)."""
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, st, en in c.execute(q):
            yield name, en - st
    else:
        import csv
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    agg = defaultdict(list)
    for name, ns in rows(sys.argv[1]):
        agg[name].append(ns)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'calls':>6} {'avg_us':>9} {'total_ms':>9} {'%':>6}  kernel")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v) / len(v) / 1e3:9.2f} {sum(v) / 1e6:9.3f} "
              f"{100 * sum(v) / tot:6.2f}  {name[:110]}")


if __name__ == "__main__":
    main()
