#!/bin/bash
# Preprocess kernel A/B: tests/test_preprocess_gpu.py, then per library
# variant of VARS (RV_LIB_VARIANT) the kernel stats of tools/time_preprocess.py
# under rocprofv3 --kernel-trace --stats, ROUNDS times.
#   TAG=x VARS="default base" bash tools/gpu_prep_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-prep}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_preprocess_gpu.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARS:-default base}; do
    d=$OUT/${v}_$r
    RV_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o tr -- \
      python3 tools/time_preprocess.py > $d.log 2>&1 || { tail $d.log; exit 1; }
    st=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$st" "$v #$r" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    for k in ("clahe_lut_kernel", "med3_kernel", "letterbox_pad"):
        if k in n:
            out.append(f"{k} {r['Calls']}x {float(r['AverageNs'])/1e3:.1f}us")
print(sys.argv[2], " | ".join(out))
PY
    rm -rf $d
  done
done
