#!/bin/bash
# r03 call 21: hardware queues per process (GPU_MAX_HW_QUEUES 4 = default / 8 / 16) with the
# native launch list; pipeline stages may be serialised behind each other's event waits when
# their streams share a queue
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --tune-save $O/tune.json > $O/q4.json 2> $O/q4.err &&
GPU_MAX_HW_QUEUES=8 $T 300 $B --tune-load $O/tune.json > $O/q8.json 2> $O/q8.err &&
GPU_MAX_HW_QUEUES=16 $T 300 $B --tune-load $O/tune.json > $O/q16.json 2> $O/q16.err &&
$T 300 $B --tune-load $O/tune.json > $O/q4b.json 2> $O/q4b.err &&
GPU_MAX_HW_QUEUES=8 $T 300 $B --tune-load $O/tune.json > $O/q8b.json 2> $O/q8b.err
rc=$?
for f in q4 q8 q16 q4b q8b; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'])"; done
exit $rc
