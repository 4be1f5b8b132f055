#!/bin/bash
# A/B one environment variable on one box: for each value, the bench line
# (autotune log on stderr with RV_CONV_DEBUG=1) and a kernel-trace breakdown
# of the graph replays.  VAR=name VALS="a b" TAG=dir bash tools/ab_env.sh
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for v in $VALS; do
  export "$VAR=$v"
  RV_CONV_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-40} \
    > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  echo "$VAR=$v $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'])")"
  [ "${SKIP_TRACE:-0}" = 1 ] && continue
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$v" -o trace -- \
    python3 tools/trace_step.py > "$OUT/trace_$v.log" 2>&1
  f=$(find "$OUT/tr_$v" -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_breakdown.py "$f" 19 > "$OUT/breakdown_$v.txt"
  rm -rf "$OUT/tr_$v"
  head -3 "$OUT/breakdown_$v.txt"
done
