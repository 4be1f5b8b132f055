"""Per-kernel-family PMC summary of one eager bench step (the passes of
tools/gpu_pmc.sh, merged by dispatch order): launches, summed counters and
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (CUs x 4 SIMDs x GRBM_GUI_ACTIVE / 8)
              (GRBM_GUI_ACTIVE sums the 8 XCDs; MICROARCH.md 'DVFS give-back')
  wait_any / wait_inst / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
              SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  read / write bytes = 2 x FETCH_SIZE, WRITE_SIZE (KB -> B; gfx950 calibration)
Usage: pmc_family.py out.json pass*.csv"""
import json
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
from pmc_report import load  # noqa: E402

CUS = 256


def family(name):
    n = name.split("(")[0].replace("void rv::", "").replace("rv::", "")
    return n.split("<")[0].strip()


def main():
    out = sys.argv[1]
    passes = [load(p) for p in sys.argv[2:]]
    n = min(len(p) for p in passes)
    fam = {}
    for i in range(n):
        v = {}
        for p in passes:
            v.update({k: x for k, x in p[i].items() if k != "name"})
        f = fam.setdefault(family(passes[0][i]["name"]), {"launches": 0})
        f["launches"] += 1
        for k, x in v.items():
            f[k] = f.get(k, 0.0) + x
    rows = {}
    for name, f in fam.items():
        r = {"launches": f["launches"]}
        wc = f.get("SQ_WAVE_CYCLES", 0.0)
        gui = f.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if gui > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in f:
            r["mfma_util"] = round(f["SQ_VALU_MFMA_BUSY_CYCLES"] / (CUS * 4 * gui), 4)
            r["gpu_cycles"] = round(gui)
        if wc > 0:
            for k, lab in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                           ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "wait_inst_lds")):
                if k in f:
                    r[lab] = round(f[k] / wc, 4)
        if f.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
            r["lds_conflict"] = round(f.get("SQ_LDS_BANK_CONFLICT", 0.0) / f["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in f:
            r["read_bytes"] = round(2 * f["FETCH_SIZE"] * 1024)
        if "WRITE_SIZE" in f:
            r["write_bytes"] = round(f["WRITE_SIZE"] * 1024)
        for k in ("SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAVES"):
            if k in f:
                r[k] = round(f[k])
        rows[name] = r
    json.dump(rows, open(out, "w"), indent=1)
    for name, r in sorted(rows.items(), key=lambda t: -t[1].get("gpu_cycles", 0)):
        print(f"{name:34s} " + " ".join(f"{k}={v}" for k, v in r.items()))


if __name__ == "__main__":
    main()
