"""Per-dispatch counters of the last bench step from rocprofv3
counter_collection.csv files (one per --pmc pass), merged by dispatch order.
Usage: pmc_report.py csv [csv ...]  -> table on stdout.  The last step starts
at the last letterbox_pad_kernel dispatch before the last clahe_lut_kernel
(or at that clahe_lut_kernel)."""
import csv
import sys
from collections import OrderedDict


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = list(disp.values())
    last = max(i for i, d in enumerate(rows) if "clahe_lut_kernel" in d["name"])
    # the fused preprocess runs one LUT launch per frame group (RV_PRE_GROUP),
    # all after the step's letterbox_pad_kernel
    pads = [i for i, d in enumerate(rows[:last]) if "letterbox_pad_kernel" in d["name"]]
    start = pads[-1] if pads else last
    return rows[start:]


def main():
    passes = [load(p) for p in sys.argv[1:]]
    n = min(len(p) for p in passes)
    cols = []
    for p in passes:
        cols += [c for c in p[0] if c != "name" and c not in cols]
    print("idx " + " ".join(f"{c[:14]:>14s}" for c in cols) + "  kernel")
    tot = {c: 0.0 for c in cols}
    for i in range(n):
        vals = {}
        for p in passes:
            vals.update({k: v for k, v in p[i].items() if k != "name"})
        for c in cols:
            tot[c] += vals.get(c, 0.0)
        name = passes[0][i]["name"].split("(")[0].replace("void rv::", "")[:40]
        print(f"{i:3d} " + " ".join(f"{vals.get(c, 0):14.0f}" for c in cols) + f"  {name}")
    print("sum " + " ".join(f"{tot[c]:14.0f}" for c in cols))


if __name__ == "__main__":
    main()
