# A/B of the Detect decode kernel: kernel-trace stats of tools/time_yolo.py
# at batch 128 per setting VARIANT:TPB (RV_LIB_VARIANT, RV_DECODE_TPB).
# usage: TAG=r04dec bash tools/decode_ab.sh base:1 default:4 default:8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-decab}
mkdir -p "$OUT"
for VT in "$@"; do
  V=${VT%%:*}; T=${VT##*:}; N="${V}_$T"
  RV_LIB_VARIANT=$V RV_DECODE_TPB=$T B=128 timeout -k 10 240 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$OUT/raw_$N" -o tr -- python3 tools/time_yolo.py > "$OUT/dec_$N.log" 2>&1 || exit $?
  ST=$(find "$OUT/raw_$N" -name "*kernel_stats.csv" | head -1)
  cp "$ST" "$OUT/stats_$N.csv"
  echo "$N $(grep -h detect_decode "$OUT/stats_$N.csv" | awk -F'",' '{print $2}' | cut -d, -f1-3)" >> "$OUT/summary.txt"
  rm -rf "$OUT/raw_$N"
done
cat "$OUT/summary.txt"
