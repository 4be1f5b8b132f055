#!/bin/bash
# r03 call 12: pipeline-shape A/B at the driver's --steps 20 (unit size, consumer on/off, run order)
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --tune-save $O/tune.json > $O/p4.json 2> $O/p4.err &&
$T 300 $B --pair 2 > $O/p2.json 2> $O/p2.err &&
$T 300 $B --pair 5 > $O/p5.json 2> $O/p5.err &&
$T 300 $B --tune-load $O/tune.json --no-consumer > $O/nc.json 2> $O/nc.err &&
RV_BENCH_DEVICE_FIRST=1 $T 300 $B --tune-load $O/tune.json > $O/df.json 2> $O/df.err &&
$T 300 $B --tune-load $O/tune.json > $O/p4b.json 2> $O/p4b.err
rc=$?
for f in p4 p2 p5 nc df p4b; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'] if 'device_only' in d else '-', d.get('steady_state_frames_per_s'))"; done
exit $rc
