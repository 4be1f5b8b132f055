#!/bin/bash
# r03 call 7: first-run effect of the native schedule (warm runs 0 / 1), with / without consumer
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
$T 300 $B --warm-runs 0 > $O/w0.json 2> $O/w0.err &&
$T 300 $B --warm-runs 1 > $O/w1.json 2> $O/w1.err &&
$T 300 $B --warm-runs 1 > $O/w1b.json 2> $O/w1b.err &&
$T 300 $B --warm-runs 1 --no-consumer > $O/w1nc.json 2> $O/w1nc.err
