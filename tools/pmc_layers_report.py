"""Per-conv-launch table from tools/pmc_layers.py's rocprofv3 --pmc passes:
the dispatches between the last two rv_trace_marker kernels (one forward),
conv-family kernels only, named from layers.json in launch order.
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x GRBM_GUI_ACTIVE / 8)
  wait_any / wait_inst / active = fractions of SQ_WAVE_CYCLES
  wait_lds    = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  lds_conf    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  read_MB     = 2 x FETCH_SIZE (KB; gfx950 calibration), write_MB = WRITE_SIZE
Usage: pmc_layers_report.py layers.json pass*.csv"""
import csv
import json
import sys
from collections import OrderedDict

FAM = ("conv_patch_kernel", "conv1x1_direct_kernel", "c2f_chain_kernel", "stem_kernel")


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = list(disp.values())
    marks = [i for i, d in enumerate(rows) if "trace_marker" in d["name"]]
    a, b = marks[-2], marks[-1]
    return [d for d in rows[a + 1:b] if any(f in d["name"] for f in FAM)]


def main():
    meta = json.load(open(sys.argv[1]))
    passes = [load(p) for p in sys.argv[2:]]
    n = min(len(p) for p in passes)
    names = meta["layers"]
    if n != len(names):
        print(f"warning: {n} conv dispatches, {len(names)} layer names")
    hdr = (f"{'layer':22s} {'kernel':14s} {'mfma':>5s} {'wany':>5s} {'winst':>5s} {'act':>5s} "
           f"{'wlds':>5s} {'v/mf':>5s} {'l/mf':>5s} {'ldsc':>5s} {'rdMB':>7s} {'wrMB':>7s} {'gui':>9s}")
    print(hdr)
    tot = {}
    for i in range(n):
        v = {}
        for p in passes:
            v.update({k: x for k, x in p[i].items() if k != "name"})
        for k, x in v.items():
            tot[k] = tot.get(k, 0.0) + x
        print(row(names[i] if i < len(names) else "?", passes[0][i]["name"], v))
    print(row("TOTAL", "", tot))


def row(name, kname, v):
    g = lambda k: v.get(k, 0.0)  # noqa: E731
    wc = g("SQ_WAVE_CYCLES") or 1.0
    gui = g("GRBM_GUI_ACTIVE")
    mf = g("SQ_INSTS_MFMA") or 1.0
    kn = kname.split("(")[0].replace("void rv::", "").replace("rv::", "")
    kn = kn.replace("conv_patch_kernel", "patch").replace("conv1x1_direct_kernel", "1x1")
    kn = kn.replace("c2f_chain_kernel", "c2f").replace("stem_kernel", "stem")
    return (f"{name:22s} {kn[:14]:14s} "
            f"{g('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * gui / 8) if gui else 0:5.3f} "
            f"{g('SQ_WAIT_ANY') / wc:5.3f} {g('SQ_WAIT_INST_ANY') / wc:5.3f} "
            f"{g('SQ_ACTIVE_INST_ANY') / wc:5.3f} {g('SQ_WAIT_INST_LDS') / wc:5.3f} "
            f"{g('SQ_INSTS_VALU') / mf:5.2f} {g('SQ_INSTS_LDS') / mf:5.2f} "
            f"{g('SQ_LDS_BANK_CONFLICT') / (g('SQ_LDS_IDX_ACTIVE') or 1):5.3f} "
            f"{2 * g('FETCH_SIZE') / 1024:7.1f} {g('WRITE_SIZE') / 1024:7.1f} {gui:9.0f}")


if __name__ == "__main__":
    main()
