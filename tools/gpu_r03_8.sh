#!/bin/bash
# r03 call 8: first-run effect: warm runs 1 / 3, device-only run first
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --warm-runs 3 > $O/w3.json 2> $O/w3.err &&
RV_BENCH_DEVICE_FIRST=1 $T 300 $B --warm-runs 1 > $O/df.json 2> $O/df.err &&
$T 300 $B --warm-runs 1 > $O/w1.json 2> $O/w1.err
