#!/bin/bash
# r03 call 19: exact-decimation letterbox copy in the fused preprocess -- preprocess/engine parity,
# then the bench line with the timed-region kernel trace
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_preprocess_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 &&
$T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing none --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err &&
TAG=r03r/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=none $T 400 bash tools/gpu_profile.sh > $O/prof.log 2>&1
rc=$?
tail -2 $O/pytest.log
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['device_only']['value'])"
cat $O/prof/timed_summary.txt
exit $rc
