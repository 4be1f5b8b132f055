#!/bin/bash
# PMC passes over one eager bench step (tools/pmc_step.py), one rocprofv3 run
# per counter group (rocprofv3 does not split groups over passes).
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
    "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
    ${EXTRA_GROUPS:-}; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 tools/pmc_step.py > "$OUT/p$i.log" 2>&1
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/pass$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 tools/pmc_report.py "$OUT"/pass*.csv > "$OUT/report.txt"
python3 tools/pmc_traffic.py "$OUT/pmc_traffic.json" "$OUT"/pass1.csv "$OUT"/pass2.csv
python3 tools/pmc_family.py "$OUT/pmc_family.json" "$OUT"/pass*.csv > "$OUT/pmc_family.txt"
rm -f "$OUT"/pass*.csv  # large (every dispatch of the run); the report keeps the last step
tail -3 "$OUT/report.txt"
