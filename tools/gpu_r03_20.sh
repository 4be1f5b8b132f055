#!/bin/bash
# r03 call 20: exact-decimation letterbox copy + compile-time head MFMA section in the decode --
# preprocess / layer / detect / engine parity, bench A/B (RV_DECODE_FIXED=0), timed-region trace
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 800 $P tests/test_preprocess_gpu.py tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 &&
$T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing none --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err &&
RV_DECODE_FIXED=0 $T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing none --tune-load $O/tune.json > $O/bench_nofix.json 2> $O/bench_nofix.err &&
TAG=r03r/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=none $T 400 bash tools/gpu_profile.sh > $O/prof.log 2>&1
rc=$?
tail -2 $O/pytest.log
for f in bench bench_nofix; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'])"; done
cat $O/prof/timed_summary.txt
exit $rc
