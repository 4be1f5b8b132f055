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
    "SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
    ${EXTRA_GROUPS:-}; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 tools/pmc_step.py > "$OUT/p$i.log" 2>&1
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/pass$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 tools/pmc_report.py "$OUT"/pass*.csv > "$OUT/report.txt"
tail -3 "$OUT/report.txt"
