#!/bin/bash
# Eager per-kernel device time of the B=128 1080p detector (tools/time_yolo.py:
# forward, NMS, letterbox+forward+NMS) under rocprofv3 --kernel-trace --stats,
# for each library variant of VARS in turn (RV_LIB_VARIANT), twice.
#   TAG=x VARS="head default" bash tools/gpu_kstats_eager.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-kse}
mkdir -p $OUT
for r in 1 2; do
  for v in ${VARS:-head default}; do
    d=$OUT/${v}_$r
    RV_LIB_VARIANT=$v B=128 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o tr -- \
      python3 tools/time_yolo.py > $d.log 2>&1 || { tail $d.log; exit 1; }
    st=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "$v #$r: $(tail -1 $d.log)"
    python3 - "$st" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    for k in ("detect_decode", "nms_kernel", "stem_kernel", "c2f_chain", "sppf"):
        if k in n:
            print(f"   {k:14s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
    rm -rf $d
  done
done
