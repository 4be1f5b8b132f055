"""Per-dispatch PMC table from a rocprofv3 counter_collection.csv: the last
`period` dispatches (one forward), counters side by side, per-wave values."""
import csv
import sys
from collections import OrderedDict


def main():
    path, period = sys.argv[1], int(sys.argv[2])
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": r["Grid_Size"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = list(disp)[-period:]
    cols = [c for c in next(iter(disp.values())) if c not in ("name", "grid")]
    print("idx grid " + " ".join(f"{c[3:15]:>12s}" for c in cols))
    for i, k in enumerate(keys):
        d = disp[k]
        w = d.get("SQ_WAVES", 1.0) or 1.0
        vals = " ".join(f"{(d.get(c, 0) / w if c != 'SQ_WAVES' else d.get(c, 0)):12.1f}" for c in cols)
        print(f"{i:3d} {d['grid']:>8s} {vals} {d['name'][13:60]}")


if __name__ == "__main__":
    main()
