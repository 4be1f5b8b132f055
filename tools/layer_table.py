"""Per-launch table of one bench step: kernel-trace duration (mean over the
graph replays of tools/trace_step.py) joined by position with the PMC passes
of tools/pmc_step.py (tools/gpu_pmc.sh) and the conv list of the plan.
Usage: layer_table.py trace.csv pass1.csv [pass2.csv ...]"""
import csv
import os
import sys
from collections import OrderedDict

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
from pmc_report import load  # noqa: E402


def step_durations(path, reps=20):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    starts = [i for i, r in enumerate(rows) if "clahe_lut_kernel" in r[2]]
    starts = starts[-reps:]
    per = starts[1] - starts[0]
    out = []
    for j in range(per):
        ds = [rows[s + j][1] - rows[s + j][0] for s in starts if s + j < len(rows)]
        out.append((rows[starts[0] + j][2], sum(ds) / len(ds) / 1e3))
    return out


def main():
    dur = step_durations(sys.argv[1])
    passes = [load(p) for p in sys.argv[2:]]
    n = min([len(dur)] + [len(p) for p in passes])
    hdr = f"{'#':>3} {'us':>7} {'rdMB':>7} {'wrMB':>7} {'GB/s':>6} {'mfma':>8} {'valu/w':>7} {'lds/w':>6} {'waves':>6} {'wcyc/w':>7} {'stall%':>6} {'wait%':>6}  kernel"
    print(hdr)
    tr = tw = tt = 0.0
    for i in range(n):
        v = {}
        for p in passes:
            v.update({k: x for k, x in p[i].items() if k != "name"})
        name, us = dur[i]
        rd = 2 * v.get("FETCH_SIZE", 0) * 1024 / 1e6
        wr = v.get("WRITE_SIZE", 0) * 1024 / 1e6
        w = max(v.get("SQ_WAVES", 1), 1)
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        tr += rd
        tw += wr
        tt += us
        print(f"{i:3d} {us:7.1f} {rd:7.1f} {wr:7.1f} {(rd + wr) / max(us, 1e-3) * 1e3:6.0f} "
              f"{v.get('SQ_INSTS_MFMA', 0):8.0f} {v.get('SQ_INSTS_VALU', 0) / w:7.0f} "
              f"{v.get('SQ_INSTS_LDS', 0) / w:6.0f} {w:6.0f} {4 * wc / w:7.0f} "
              f"{100 * v.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {100 * v.get('SQ_WAIT_ANY', 0) / wc:6.1f}  "
              f"{name.split('(')[0].replace('void rv::', '')[:44]}")
    print(f"tot {tt:7.1f} {tr:7.1f} {tw:7.1f}")


if __name__ == "__main__":
    main()
