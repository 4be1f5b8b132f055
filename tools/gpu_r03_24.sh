#!/bin/bash
# r03 call 24: fused one-launch SORT step -- SORT / engine parity; bench A/B (RV_SORT_FUSED=0),
# Detect-head side streams on / off, high-priority preprocess stream
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_sort_gpu.py tests/test_track_ops_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --tune-save $O/tune.json > $O/fused1.json 2> $O/fused1.err || exit 1
RV_SORT_FUSED=0 $T 300 $B --tune-load $O/tune.json > $O/three1.json 2> $O/three1.err || exit 1
$T 300 $B --tune-load $O/tune.json > $O/fused2.json 2> $O/fused2.err || exit 1
RV_SORT_FUSED=0 $T 300 $B --tune-load $O/tune.json > $O/three2.json 2> $O/three2.err || exit 1
RV_HEAD_STREAMS=0 $T 300 $B --tune-load $O/tune.json > $O/hs0_1.json 2> $O/hs0_1.err || exit 1
RV_HEAD_STREAMS=0 $T 300 $B --tune-load $O/tune.json > $O/hs0_2.json 2> $O/hs0_2.err || exit 1
RV_PREP_PRIORITY=-1 $T 300 $B --tune-load $O/tune.json > $O/prio.json 2> $O/prio.err || exit 1
RV_CONSUMER_DEFER=1 $T 300 $B --tune-load $O/tune.json > $O/defer.json 2> $O/defer.err || exit 1
RV_CONSUMER_NOGC=1 $T 300 $B --tune-load $O/tune.json > $O/nogc.json 2> $O/nogc.err || exit 1
tail -2 $O/pytest.log
for f in fused1 three1 fused2 three2 hs0_1 hs0_2 prio defer nogc; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'])"; done
