"""HBM traffic of the conv launches (conv_patch_kernel + conv1x1_direct_kernel +
c2f_chain_kernel + stem_kernel)
of one bench step from the PMC
passes of tools/gpu_pmc.sh (FETCH_SIZE / WRITE_SIZE, KB): per the gfx950
calibration in MI355X_MICROARCH.md, FETCH_SIZE counts half the bytes of a
wide streaming read (x2), WRITE_SIZE counts 16-B-per-lane stores exactly.
Writes a JSON file that bench.py reports as roofline.traffic.
Usage: pmc_traffic.py out.json pass1.csv pass2.csv ..."""
import hashlib
import json
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
from pmc_report import load  # noqa: E402

CONV_KERNELS = ("conv_patch_kernel", "conv1x1_direct_kernel", "c2f_chain_kernel", "stem_kernel")


def main():
    out = sys.argv[1]
    passes = [load(p) for p in sys.argv[2:]]
    n = min(len(p) for p in passes)
    fetch = write = 0.0
    per_kernel = {}
    for i in range(n):
        v = {}
        for p in passes:
            v.update({k: x for k, x in p[i].items() if k != "name"})
        name = passes[0][i]["name"].split("(")[0].replace("void rv::", "").replace("rv::", "")
        rd = 2 * v.get("FETCH_SIZE", 0.0) * 1024
        wr = v.get("WRITE_SIZE", 0.0) * 1024
        k = per_kernel.setdefault(name.split("<")[0], [0, 0.0, 0.0])
        k[0] += 1
        k[1] += rd
        k[2] += wr
        if name.startswith(CONV_KERNELS):
            fetch += rd
            write += wr
    unit = int(os.environ.get("PAIR", 4))  # steps per profiled forward (tools/pmc_step.py)
    fetch, write = fetch / unit, write / unit
    res = {"conv_bytes_per_step": fetch + write, "conv_read_bytes": fetch,
           "conv_write_bytes": write, "conv_kernels": list(CONV_KERNELS),
           "steps_per_forward": unit,
           # the library the counters were collected on: bench.py reports this
           # traffic only while the same build is loaded
           "librvhip_sha256": hashlib.sha256(open(os.path.join(
               os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
               "road-vision-system_amd", "rvs_amd", "librvhip.so"), "rb").read()).hexdigest(),
           "per_kernel": {k: {"launches": c, "read_bytes": r, "write_bytes": w}
                          for k, (c, r, w) in per_kernel.items()},
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over one eager pipeline "
                     "unit (tools/gpu_pmc.sh, tools/pmc_step.py: one forward over PAIR steps' "
                     "frames, conv bytes / PAIR per step); read = 2 x FETCH_SIZE (gfx950 "
                     "calibration), KB -> B"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))


if __name__ == "__main__":
    main()
