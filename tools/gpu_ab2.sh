#!/bin/bash
# Interleaved A/B of environment switches on one box, each run autotuned on
# its own (the switch can change which conv configuration wins): optional
# GPU tests first, then ROUNDS x every "label;env assignments" of CONFIGS:
# the driver's bench (--steps 20, no CPU baseline / secondary legs) and, with
# CONV=1, the eager per-conv table (tools/conv_profile.py, B = 128).
#   TAG=x TESTS="tests/test_sort_gpu.py" CONFIGS=$'a;RV_X=0\nb;RV_X=1' bash tools/gpu_ab2.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab2}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
  tail -n 1 $OUT/pytest.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  while IFS=';' read -r label envs; do
    [ -z "$label" ] && continue
    f=$OUT/${label}_$r.json
    env $envs timeout -k 10 400 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline \
      --no-secondary $BENCH_ARGS > $f 2> ${f%.json}.err || { tail -n 30 ${f%.json}.err; exit 1; }
    echo "$label #$r: $(python3 -c "
import json;d=json.load(open('$f'))
r=d.get('roofline') or {}
print(d['value'], d['ms_per_step'], 'steady', d.get('steady_state_frames_per_s'), 'conv_union', r.get('conv_ms_per_step'), 'eager', (r.get('eager') or {}).get('frac'))")"
    if [ "${CONV:-0}" = 1 ] && [ "$r" = 1 ]; then
      env $envs B=128 timeout -k 10 300 python -u tools/conv_profile.py > $OUT/conv_${label}.log 2>&1 || exit 1
      echo "  $(grep 'conv sum' $OUT/conv_${label}.log)"
    fi
  done <<< "$CONFIGS"
done
