#!/bin/bash
# r03 call 18: every autotune candidate's time (RV_CONV_DEBUG=2)
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
export PYTHONUNBUFFERED=1
RV_CONV_DEBUG=2 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --conv-timing none > $O/bench.json 2> $O/bench.err
rc=$?
grep autotune $O/bench.err > $O/autotune_all.txt
grep -c cand $O/autotune_all.txt
exit $rc
