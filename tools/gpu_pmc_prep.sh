#!/bin/bash
# PMC passes over tools/prep_pmc_run.py (fused preprocess only), one
# rocprofv3 run per counter group; summary per kernel family.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmc_prep}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
    "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 tools/prep_pmc_run.py > "$OUT/p$i.log" 2>&1
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/pass$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 tools/pmc_family.py "$OUT/pmc_family.json" "$OUT"/pass*.csv > "$OUT/pmc_family.txt"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for p in sorted(glob.glob(out + "/pass*.csv")):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void rv::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
with open(out + "/raw_totals.txt", "w") as f:
    for k, c in tot.items():
        f.write(k + "\n" + "".join(f"  {n} {v:.0f}\n" for n, v in sorted(c.items())))
PY
rm -f "$OUT"/pass*.csv
cat "$OUT/pmc_family.txt"
