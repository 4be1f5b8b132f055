#!/bin/bash
# Interleaved bench A/B on one box at the driver's size (--steps 20): each
# configuration "label;env assignments;bench args" of CONFIGS (newline
# separated) runs ROUNDS times in turn; conv configurations are autotuned
# once and loaded by every run.  TAG=x CONFIGS=$'even;;\nramp;;--units ramp' bash tools/gpu_bench_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-bab}
mkdir -p "$OUT"
STEPS=${STEPS:-20}
COMMON="--gpus 1 --steps $STEPS --warmup 5 --no-cpu-baseline --no-secondary --conv-timing none"
timeout -k 10 400 python -u bench.py $COMMON --tune-save $OUT/tune.json > $OUT/tune_run.json 2> $OUT/tune_run.err \
  || { tail -n 30 $OUT/tune_run.err; exit 1; }
echo "tune run: $(python3 -c "import json;d=json.load(open('$OUT/tune_run.json'));print(d['value'], d['ms_per_step'])")"
for r in $(seq 1 ${ROUNDS:-2}); do
  while IFS=';' read -r label envs args; do
    [ -z "$label" ] && continue
    f=$OUT/${label}_$r.json
    env $envs timeout -k 10 400 python -u bench.py $COMMON --tune-load $OUT/tune.json $args > $f 2> ${f%.json}.err \
      || { tail -n 30 ${f%.json}.err; exit 1; }
    echo "$label #$r: $(python3 -c "
import json;d=json.load(open('$f'))
print(d['value'], d['ms_per_step'], (d.get('device_only') or {}).get('value'), d.get('steady_state_frames_per_s'))")"
  done <<< "$CONFIGS"
done
