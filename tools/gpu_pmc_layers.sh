#!/bin/bash
# Per-conv-launch PMC table of one B = 128 forward (tools/pmc_layers.py):
# an unprofiled run saves the tuned configurations and the launch names,
# then one rocprofv3 --pmc pass per counter group.  TAG=x [RV_LIB_VARIANT=v]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmcl}
mkdir -p "$OUT"
timeout -k 10 300 env TUNE_SAVE=$OUT/tune.json LAYERS=$OUT/layers.json python3 tools/pmc_layers.py \
  > "$OUT/prep.log" 2>&1 || { tail -n 20 "$OUT/prep.log"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
    "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  TUNE=$OUT/tune.json timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 tools/pmc_layers.py > "$OUT/p$i.log" 2>&1 || { tail -n 20 "$OUT/p$i.log"; exit 1; }
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/pass$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 tools/pmc_layers_report.py "$OUT/layers.json" "$OUT"/pass*.csv > "$OUT/pmc_layers.txt"
rm -f "$OUT"/pass*.csv
cat "$OUT/pmc_layers.txt"
