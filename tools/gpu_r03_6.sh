#!/bin/bash
# r03 call 6: bench with the C Detection builder (steps 20 / 60), then the nested-capture
# repro (pure HIP, no torch): control, re-used events, fresh events.  A crash ends the call.
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python bench.py --steps 20 --no-cpu-baseline --conv-timing none > $O/bench20.json 2> $O/bench20.err &&
$T 400 python bench.py --steps 60 --no-cpu-baseline --conv-timing none > $O/bench60.json 2> $O/bench60.err &&
$T 60 tools/repro_nested_capture 0 8 400 > $O/repro0.log 2>&1 &&
$T 60 tools/repro_nested_capture 2 8 400 > $O/repro2.log 2>&1 &&
$T 60 tools/repro_nested_capture 1 8 400 > $O/repro1.log 2>&1
