#!/bin/bash
# r03 call 23: Detect-head side streams (they share a hardware queue with the preprocess stream:
# rocprof Queue_Id) on / off, and a high-priority preprocess stream; interleaved repeats
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --tune-save $O/tune.json > $O/base1.json 2> $O/base1.err || exit 1
for i in 2 3; do
  RV_HEAD_STREAMS=0 $T 300 $B --tune-load $O/tune.json > $O/hs0_$i.json 2> $O/hs0_$i.err || exit 1
  $T 300 $B --tune-load $O/tune.json > $O/base$i.json 2> $O/base$i.err || exit 1
done
RV_PREP_PRIORITY=-1 $T 300 $B --tune-load $O/tune.json > $O/prio.json 2> $O/prio.err &&
RV_HEAD_STREAMS=0 RV_PREP_PRIORITY=-1 $T 300 $B --tune-load $O/tune.json > $O/hs0prio.json 2> $O/hs0prio.err
rc=$?
for f in base1 hs0_2 base2 hs0_3 base3 prio hs0prio; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'])"; done
exit $rc
