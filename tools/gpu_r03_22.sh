#!/bin/bash
# r03 call 22: fewer streams per pipeline -- Detect heads on the Y2 stream (RV_HEAD_STREAMS=0),
# the track stage on the Y2 stream (RV_TRACK_ON_Y2=1), both
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --tune-save $O/tune.json > $O/base.json 2> $O/base.err &&
RV_HEAD_STREAMS=0 $T 300 $B --tune-load $O/tune.json > $O/hs0.json 2> $O/hs0.err &&
RV_TRACK_ON_Y2=1 $T 300 $B --tune-load $O/tune.json > $O/ty2.json 2> $O/ty2.err &&
RV_HEAD_STREAMS=0 RV_TRACK_ON_Y2=1 $T 300 $B --tune-load $O/tune.json > $O/both.json 2> $O/both.err &&
$T 300 $B --tune-load $O/tune.json > $O/base2.json 2> $O/base2.err
rc=$?
for f in base hs0 ty2 both base2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'])"; done
exit $rc
